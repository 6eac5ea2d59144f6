// 1x1-only convolution jobs as a plain tiled GEMM on gfx950 f32 MFMA.
//
// Replaces the 1x1 convs of the training path whose only segments are pointwise:
// SpectralTransform.conv1 / conv2 (layers/ffc/spectral_transform.py:52-53,70-71,89,108), the
// Fourier unit's spectral mix conv_layer (layers/ffc/fourier_unity.py:25,45) applied to the
// interleaved (B, 2C, H, W/2+1) spectrum, and the adjoints (data gradients) of all of them.
// On the LDS-patch kernel a 1x1 segment multiplies one 16-deep k group per staged chunk and
// shares each staged input element across only 32 output channels; here a workgroup owns a
// BM x BN tile (BM up to 128 output channels) and K (all segments' channels) runs in 32-deep
// chunks through padded LDS, with the next chunk's loads in registers under the MFMAs.
//
//   out[b][m][q] = act( sum_s sum_c A[m][k(s, c)] * x_s[b][c][q]  + bias[m] + addend[b][m][q] )
//
// n = b * Q + q (Q = OH * OW, the same for every segment).  A is the packed [Mpad][Kpad] weight
// of a one-phase ffc_conv_job (k = segment-major channel index, ffc_conv_pack).  v_mfma_f32_32x32x2_f32:
// exact fp32 products, fp32 accumulation.
#include "ffc_internal.h"

namespace {

constexpr int PW_BK = 32;

struct PwArgs {
    const float* x[FFC_MAX_SEG];
    int cend[FFC_MAX_SEG];   // cumulative channel count: segment s owns k in [cend[s-1], cend[s])
    int nseg;
    const float* A;
    int Kpad;
    float* out;
    const float* bias;
    const float* addend;
    int B, M, Q, K, ntn;
    int act;
    float act_param;
};

template <int BM, int BN>
__global__ __launch_bounds__(256) void pw_gemm_kernel(PwArgs a) {
    constexpr int LDA = PW_BK + 1;           // conflict-free column reads of A
    constexpr int LDB = BN + 32;             // rows 2s and 2s+1 of a k-step land 32 banks apart
    constexpr int WTM = BM / 2, WTN = BN / 2;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int APT = BM * PW_BK / 256;    // A floats per thread per chunk (8 or 16)
    constexpr int ATR = PW_BK / APT;         // threads per A row
    constexpr int BG = 256 / BN;             // k groups of B staging
    constexpr int BPT = PW_BK / BG;          // B floats per thread per chunk
    __shared__ __attribute__((aligned(16))) float As[BM * LDA];
    __shared__ __attribute__((aligned(16))) float Bs[PW_BK * LDB];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, cl = lane & 31;
    const int wm = (wave >> 1) * WTM, wn = (wave & 1) * WTN;
    const int tn = blockIdx.x % a.ntn, tm = blockIdx.x / a.ntn;
    const int m0 = tm * BM, n0 = tn * BN;
    const int N = a.B * a.Q;

    // A staging: row ar, k offset ak of every chunk
    const int ar = tid / ATR, ak = (tid % ATR) * APT;
    const float* __restrict__ Arow = a.A + (size_t)(m0 + ar) * a.Kpad + ak;
    // B staging: one pixel n per thread (coalesced along q), a wave-uniform k group
    const int bn = tid % BN;
    const int bg = __builtin_amdgcn_readfirstlane(tid / BN);
    const int nn = n0 + bn;
    const bool nok = nn < N;
    const int b = nok ? nn / a.Q : 0;
    const int q = nok ? nn - b * a.Q : 0;

    floatx4 ra[APT / 4];
    float rb[BPT];
    auto load = [&](int k0) {
#pragma unroll
        for (int i = 0; i < APT / 4; ++i)
            ra[i] = (k0 + ak + 4 * i < a.Kpad) ? *reinterpret_cast<const floatx4*>(Arow + k0 + 4 * i)
                                               : floatx4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int j = 0; j < BPT; ++j) {
            const int k = k0 + bg * BPT + j;   // wave-uniform
            float v = 0.0f;
            if (k < a.K && nok) {
                // segment select chains on kernel arguments (no dynamically indexed argument arrays)
                const bool s0 = k < a.cend[0], s1 = !s0 && k < a.cend[1];
                const float* xs = s0 ? a.x[0] : (s1 ? a.x[1] : a.x[2]);
                const int c0 = s0 ? 0 : (s1 ? a.cend[0] : a.cend[1]);
                const int C = (s0 ? a.cend[0] : (s1 ? a.cend[1] : a.cend[2])) - c0;
                v = xs[((size_t)b * C + (k - c0)) * a.Q + q];
            }
            rb[j] = v;
        }
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

    load(0);
    for (int k0 = 0; k0 < a.Kpad; k0 += PW_BK) {
        __syncthreads();   // everyone is done reading the previous chunk
#pragma unroll
        for (int i = 0; i < APT / 4; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) As[ar * LDA + ak + 4 * i + e] = ra[i][e];
#pragma unroll
        for (int j = 0; j < BPT; ++j) Bs[(bg * BPT + j) * LDB + bn] = rb[j];
        __syncthreads();
        if (k0 + PW_BK < a.Kpad) load(k0 + PW_BK);   // in flight under this chunk's MFMAs
#pragma unroll
        for (int st = 0; st < PW_BK / 2; ++st) {
            float xv[TM], yv[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) xv[i] = As[(wm + 32 * i + cl) * LDA + 2 * st + h];
#pragma unroll
            for (int j = 0; j < TN; ++j) yv[j] = Bs[(2 * st + h) * LDB + wn + 32 * j + cl];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(xv[i], yv[j], acc[i][j], 0, 0, 0);
        }
    }

#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn + 32 * j + cl;
        if (n >= N) continue;
        const int ob = n / a.Q, oq = n - ob * a.Q;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (m >= a.M) continue;
                const size_t o = ((size_t)ob * a.M + m) * a.Q + oq;
                float v = acc[i][j][r];
                if (a.bias) v += a.bias[m];
                if (a.addend) v += a.addend[o];
                a.out[o] = ffc::apply_act(v, a.act, a.act_param);
            }
    }
}

constexpr int PW_TILES[3][2] = {{128, 128}, {64, 128}, {64, 64}};

}  // namespace

extern "C" int ffc_pw_tiles(int M, int B, int Q, int cfg) {
    if (cfg < 0 || cfg > 2 || M <= 0 || B <= 0 || Q <= 0) return -1;
    const long long N = (long long)B * Q;
    return (int)(((M + PW_TILES[cfg][0] - 1) / PW_TILES[cfg][0]) * ((N + PW_TILES[cfg][1] - 1) / PW_TILES[cfg][1]));
}

extern "C" int ffc_pw_forward(const ffc_conv_job* job, int cfg, void* stream) {
    FFC_CHECK_ARG(job && cfg >= 0 && cfg <= 2, "ffc_pw_forward: bad args");
    const ffc_conv_job& J = *job;
    FFC_CHECK_ARG(J.A && J.out && J.B > 0 && J.M > 0 && J.nphase == 1, "ffc_pw_forward: incomplete job");
    FFC_CHECK_ARG(J.nseg >= 1 && J.nseg <= FFC_MAX_SEG, "ffc_pw_forward: nseg out of range");
    FFC_CHECK_ARG(J.Mpad % 128 == 0 && J.Mpad >= J.M, "ffc_pw_forward: Mpad must be a multiple of 128");
    FFC_CHECK_ARG(J.ph[0].Kpad % 16 == 0 && J.ph[0].a_off == 0, "ffc_pw_forward: packed weight layout");
    FFC_CHECK_ARG(!J.stats, "ffc_pw_forward: BN partials are not produced here");
    PwArgs a{};
    int k = 0;
    for (int s = 0; s < FFC_MAX_SEG; ++s) {
        if (s < J.nseg) {
            const ffc_conv_seg& S = J.seg[s];
            FFC_CHECK_ARG(S.x && !S.pool && !S.gate && S.IH == J.OH && S.IW == J.OW && S.mult_y == 1 &&
                              S.mult_x == 1 && S.C > 0,
                          "ffc_pw_forward: segments must be 1x1 at the output resolution");
            a.x[s] = S.x;
            k += S.C;
        }
        a.cend[s] = k;
    }
    FFC_CHECK_ARG(J.ph[0].K == k && J.ph[0].Kpad >= k, "ffc_pw_forward: K");
    a.nseg = J.nseg;
    a.A = J.A;
    a.Kpad = J.ph[0].Kpad;
    a.out = J.out;
    a.bias = J.bias;
    a.addend = J.addend;
    a.B = J.B;
    a.M = J.M;
    a.Q = J.OH * J.OW;
    a.K = k;
    a.act = J.act;
    a.act_param = J.act_param;
    const long long N = (long long)a.B * a.Q;
    FFC_CHECK_ARG(N < (1LL << 31) / 2, "ffc_pw_forward: too many pixels");
    const int BM = PW_TILES[cfg][0], BN = PW_TILES[cfg][1];
    a.ntn = (int)((N + BN - 1) / BN);
    const int ntiles = ffc_pw_tiles(J.M, J.B, a.Q, cfg);
    hipStream_t s = (hipStream_t)stream;
    switch (cfg) {
        case 0: hipLaunchKernelGGL((pw_gemm_kernel<128, 128>), dim3(ntiles), dim3(256), 0, s, a); break;
        case 1: hipLaunchKernelGGL((pw_gemm_kernel<64, 128>), dim3(ntiles), dim3(256), 0, s, a); break;
        default: hipLaunchKernelGGL((pw_gemm_kernel<64, 64>), dim3(ntiles), dim3(256), 0, s, a); break;
    }
    (void)BM;
    return ffc::launch_status("ffc_pw_forward");
}
