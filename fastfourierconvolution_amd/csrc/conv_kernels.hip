// Implicit-GEMM convolution / transposed convolution on gfx950 f32 MFMA.
//
// Replaces the local-branch nn.Conv2d / nn.ConvTranspose2d of FFC / FFCTranspose
// (layers/ffc/ffc.py:45-70, layers/ffc/ffc_transpose.py:48-86) and the 1x1 conv1/conv2 of
// SpectralTransform (layers/ffc/spectral_transform.py:52-53,70-71).  Several convolutions
// that are summed into one output (convl2l(x_l)+convg2l(x_g); convl2g(x_l)+conv2(v)) are
// one GEMM whose K runs over all segments, so the sum never touches HBM.
//
// Per workgroup: a BMxBN output tile of one phase (all output pixels of a phase share one
// tap set); K in 16-deep chunks, A (pre-packed weights) and B (gathered activations) staged
// through double-buffered, padded LDS (row stride 20 floats: conflict-free ds_read_b128);
// v_mfma_f32_32x32x2_f32 (exact fp32, fmaf-chain numerics).  Lane half h = lane>>5 of k-step s
// carries logical k = 8h + s, so each lane reads its 8 k-values of a chunk as 2x b128.
// Epilogue: bias + addend, optional BN partials {n, mean, M2} per (wave, channel),
// activation, store.
#include "ffc_internal.h"

namespace {

constexpr int BK = 16;
constexpr int LDK = BK + 4;

struct ConvArgs {
    ffc_conv_job jobs[2];
    const int4* tiles;
};

template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(256) void conv_gemm_kernel(ConvArgs args_byval) {
    // Read the descriptors straight from the kernarg segment (scalar loads with a dynamic job
    // index); touching the by-value parameter would copy the whole struct to scratch.
#if defined(__HIP_DEVICE_COMPILE__)
    const ConvArgs& args = *(const ConvArgs*)__builtin_amdgcn_kernarg_segment_ptr();
#else
    const ConvArgs& args = args_byval;  // host pass only parses the body
#endif
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int A_F4 = BM * (BK / 4);
    constexpr int A_PER_T = (A_F4 + 255) / 256;
    constexpr int QPT = BN / 64;        // 4-deep k quads per thread for the B tile
    constexpr int QSTEP = 256 / BN;
    static_assert(WM * WN == 4, "4 waves");
    __shared__ __attribute__((aligned(16))) float As[2][BM * LDK];
    __shared__ __attribute__((aligned(16))) float Bs[2][BN * LDK];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int4 tile = args.tiles[blockIdx.x];
    const int jx = __builtin_amdgcn_readfirstlane(tile.x);
    const int m0 = __builtin_amdgcn_readfirstlane(tile.y);
    const int n0 = __builtin_amdgcn_readfirstlane(tile.z);
    const int slot = __builtin_amdgcn_readfirstlane(tile.w);
    const ffc_conv_job& J = args.jobs[jx & 0xff];
    const ffc_conv_phase& P = J.ph[jx >> 8];
    const int Kpad = P.Kpad;
    const int nchunks = Kpad / BK;
    const float* __restrict__ Ap = J.A + P.a_off + (size_t)m0 * Kpad;
    const int4* __restrict__ kt = reinterpret_cast<const int4*>(J.ktab) + P.kt_off;
    const int PW = P.PW;
    const int PHW = P.PH * PW;
    const int NPH = J.B * PHW;

    // B-loader geometry: this thread gathers column nl for quads qb, qb+QSTEP, ...
    const int nl = tid % BN;
    const int qb = __builtin_amdgcn_readfirstlane(tid / BN);
    const int nglob = n0 + nl;
    const bool nvalid = nglob < NPH;
    int gb = 0, gy = 0, gx = 0;
    if (nvalid) {
        gb = nglob / PHW;
        const int r = nglob - gb * PHW;
        gy = r / PW;
        gx = r - gy * PW;
    }

    static_assert(A_PER_T <= 2, "A staging uses at most two float4 per thread");
    float4 areg0 = make_float4(0.f, 0.f, 0.f, 0.f), areg1 = areg0;
    float breg[QPT][4];
    const bool a_on0 = tid < A_F4;
    const float* __restrict__ Ap0 = Ap + (size_t)(tid >> 2) * Kpad + (tid & 3) * 4;
    const float* __restrict__ Ap1 = Ap + (size_t)((tid + 256) >> 2) * Kpad + (tid & 3) * 4;

    auto load_a = [&](int chunk) {
        if (a_on0) areg0 = *reinterpret_cast<const float4*>(Ap0 + chunk * BK);
        if constexpr (A_PER_T == 2) areg1 = *reinterpret_cast<const float4*>(Ap1 + chunk * BK);
    };
    auto load_b = [&](int chunk) {
#pragma unroll
        for (int j = 0; j < QPT; ++j) {
            const int q = qb + j * QSTEP;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int k = chunk * BK + q * 4 + e;
                const int4 ent = kt[k];
                const int seg = ent.x & 15;
                float v = 0.0f;
                if (seg < FFC_MAX_SEG && nvalid) {
                    const ffc_conv_seg& S = J.seg[seg];
                    const int ch = ent.x >> 4;
                    const int iy = gy * S.mult_y + ent.y;
                    const int ix = gx * S.mult_x + ent.z;
                    if ((unsigned)iy < (unsigned)S.IH && (unsigned)ix < (unsigned)S.IW) {
                        if (!S.pool) {
                            v = S.x[(((size_t)gb * S.C + ch) * S.IH + iy) * S.IW + ix];
                        } else {
                            const int W2 = 2 * S.IW;
                            const float* p = S.x + (((size_t)gb * S.C + ch) * (2 * S.IH) + 2 * iy) * W2 + 2 * ix;
                            v = (((p[0] + p[1]) + p[W2]) + p[W2 + 1]) * 0.25f;
                        }
                        if (S.gate) v *= S.gate[(size_t)gb * S.C + ch];
                    }
                }
                breg[j][e] = v;
            }
        }
    };
    auto store_tiles = [&](int buf) {
        if (a_on0) *reinterpret_cast<float4*>(&As[buf][(tid >> 2) * LDK + (tid & 3) * 4]) = areg0;
        if constexpr (A_PER_T == 2)
            *reinterpret_cast<float4*>(&As[buf][((tid + 256) >> 2) * LDK + (tid & 3) * 4]) = areg1;
#pragma unroll
        for (int j = 0; j < QPT; ++j) {
            const int q = qb + j * QSTEP;
            *reinterpret_cast<float4*>(&Bs[buf][nl * LDK + q * 4]) =
                make_float4(breg[j][0], breg[j][1], breg[j][2], breg[j][3]);
        }
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

    const int h = lane >> 5, cl = lane & 31;
    load_a(0);
    load_b(0);
    store_tiles(0);
    __syncthreads();
    for (int c = 0; c < nchunks; ++c) {
        const int cur = c & 1;
        const bool more = c + 1 < nchunks;
        if (more) {
            load_a(c + 1);
            load_b(c + 1);
        }
        float af[TM][8], bf[TN][8];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const float* src = &As[cur][(wm * WTM + i * 32 + cl) * LDK + h * 8];
            const float4 x0 = *reinterpret_cast<const float4*>(src);
            const float4 x1 = *reinterpret_cast<const float4*>(src + 4);
            af[i][0] = x0.x; af[i][1] = x0.y; af[i][2] = x0.z; af[i][3] = x0.w;
            af[i][4] = x1.x; af[i][5] = x1.y; af[i][6] = x1.z; af[i][7] = x1.w;
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const float* src = &Bs[cur][(wn * WTN + j * 32 + cl) * LDK + h * 8];
            const float4 x0 = *reinterpret_cast<const float4*>(src);
            const float4 x1 = *reinterpret_cast<const float4*>(src + 4);
            bf[j][0] = x0.x; bf[j][1] = x0.y; bf[j][2] = x0.z; bf[j][3] = x0.w;
            bf[j][4] = x1.x; bf[j][5] = x1.y; bf[j][6] = x1.z; bf[j][7] = x1.w;
        }
#pragma unroll
        for (int s = 0; s < 8; ++s)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
        if (more) store_tiles(cur ^ 1);
        __syncthreads();
    }

    // ---------------- epilogue
    const size_t plane = (size_t)J.OH * J.OW;
    int ob[TN], oo[TN];
    bool ov[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int nn = n0 + wn * WTN + j * 32 + cl;
        ov[j] = nn < NPH;
        ob[j] = 0;
        oo[j] = 0;
        if (ov[j]) {
            const int b = nn / PHW;
            const int r = nn - b * PHW;
            const int my = r / PW, mx = r - my * PW;
            ob[j] = b;
            oo[j] = (my * J.Sy + P.py) * J.OW + (mx * J.Sx + P.px);
        }
    }
    const int mbase = m0 + wm * WTM + 4 * h;
    if (J.bias || J.addend) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = mbase + i * 32 + (r & 3) + 8 * (r >> 2);
                if (m >= J.M) continue;
                const float bv = J.bias ? J.bias[m] : 0.0f;
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    float v = acc[i][j][r] + bv;
                    if (J.addend && ov[j]) v += J.addend[((size_t)ob[j] * J.M + m) * plane + oo[j]];
                    acc[i][j][r] = v;
                }
            }
    }
    if (J.stats) {
        float cntl = 0.0f;
#pragma unroll
        for (int j = 0; j < TN; ++j) cntl += ov[j] ? 1.0f : 0.0f;
        const float cnt = ffc::half_wave_sum(cntl);
        float4* st = reinterpret_cast<float4*>(J.stats) + ((size_t)slot * WN + wn) * J.M;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = mbase + i * 32 + (r & 3) + 8 * (r >> 2);
                float s = 0.0f;
#pragma unroll
                for (int j = 0; j < TN; ++j) s += ov[j] ? acc[i][j][r] : 0.0f;
                const float mean = cnt > 0.0f ? ffc::half_wave_sum(s) / cnt : 0.0f;
                float q = 0.0f;
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const float d = ov[j] ? acc[i][j][r] - mean : 0.0f;
                    q += d * d;
                }
                const float m2 = ffc::half_wave_sum(q);
                if (cl == 0 && m < J.M) st[m] = make_float4(cnt, mean, m2, 0.0f);
            }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = mbase + i * 32 + (r & 3) + 8 * (r >> 2);
            if (m >= J.M) continue;
#pragma unroll
            for (int j = 0; j < TN; ++j)
                if (ov[j])
                    J.out[((size_t)ob[j] * J.M + m) * plane + oo[j]] =
                        ffc::apply_act(acc[i][j][r], J.act, J.act_param);
        }
}

struct PackArgs {
    ffc_conv_job job;
    const float* w[FFC_MAX_SEG];
    const float* bias[FFC_MAX_SEG];
    int layout[FFC_MAX_SEG], kh[FFC_MAX_SEG], kw[FFC_MAX_SEG];
    float* A;
    float* bias_out;
    long long total;
};

__global__ void conv_pack_kernel(PackArgs a) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const ffc_conv_job& J = a.job;
    if (idx < J.M && a.bias_out) {
        float s = 0.0f;
        for (int sg = 0; sg < J.nseg; ++sg)
            if (a.bias[sg]) s += a.bias[sg][idx];
        a.bias_out[idx] = s;
    }
    if (idx >= a.total) return;
    long long rem = idx;
    int p = 0;
    for (; p < J.nphase; ++p) {
        const long long sz = (long long)J.Mpad * J.ph[p].Kpad;
        if (rem < sz) break;
        rem -= sz;
    }
    const ffc_conv_phase& P = J.ph[p];
    const int m = (int)(rem / P.Kpad), k = (int)(rem - (long long)m * P.Kpad);
    float v = 0.0f;
    if (m < J.M && k < P.K) {
        const int4 ent = reinterpret_cast<const int4*>(J.ktab)[P.kt_off + k];
        const int sg = ent.x & 15;
        if (sg < FFC_MAX_SEG) {
            const int ch = ent.x >> 4;
            const int ky = ent.w & 0xffff, kx = ent.w >> 16;
            const int C = J.seg[sg].C;
            const int kh = a.kh[sg], kw = a.kw[sg];
            const size_t off = a.layout[sg] == 0 ? (((size_t)m * C + ch) * kh + ky) * kw + kx
                                                 : (((size_t)ch * J.M + m) * kh + ky) * kw + kx;
            v = a.w[sg][off];
        }
    }
    a.A[P.a_off + (long long)m * P.Kpad + k] = v;
}

template <int BM, int BN, int WM, int WN>
int launch_cfg(const ConvArgs& args, int ntiles, hipStream_t s) {
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, WM, WN>), dim3(ntiles), dim3(256), 0, s, args);
    return ffc::launch_status("ffc_conv_forward");
}

}  // namespace

extern "C" int ffc_conv_stat_rows_per_tile(int tile_cfg) {
    switch (tile_cfg) {
        case 0: return 2;
        case 1: return 2;
        case 2: return 4;
    }
    return 0;
}

extern "C" int ffc_conv_forward(const ffc_conv_job* jobs, int njobs, const int* tiles, int ntiles, int tile_cfg,
                                void* stream) {
    FFC_CHECK_ARG(jobs && tiles && njobs >= 1 && njobs <= 2 && ntiles > 0, "ffc_conv_forward: bad args");
    for (int j = 0; j < njobs; ++j) {
        const ffc_conv_job& J = jobs[j];
        FFC_CHECK_ARG(J.A && J.ktab && J.out && J.B > 0 && J.M > 0, "ffc_conv_forward: incomplete job");
        FFC_CHECK_ARG(J.nseg >= 1 && J.nseg <= FFC_MAX_SEG, "ffc_conv_forward: nseg out of range");
        FFC_CHECK_ARG(J.nphase >= 1 && J.nphase <= FFC_MAX_PHASE, "ffc_conv_forward: nphase out of range");
        FFC_CHECK_ARG(J.Mpad % 128 == 0 && J.Mpad >= J.M, "ffc_conv_forward: Mpad must be a multiple of 128");
        for (int p = 0; p < J.nphase; ++p)
            FFC_CHECK_ARG(J.ph[p].Kpad % BK == 0 && J.ph[p].Kpad >= J.ph[p].K && J.ph[p].Kpad > 0,
                          "ffc_conv_forward: Kpad must be a positive multiple of 16");
        for (int s = 0; s < J.nseg; ++s) FFC_CHECK_ARG(J.seg[s].x != nullptr, "ffc_conv_forward: null segment");
    }
    ConvArgs args;
    args.jobs[0] = jobs[0];
    args.jobs[1] = jobs[njobs > 1 ? 1 : 0];
    args.tiles = reinterpret_cast<const int4*>(tiles);
    hipStream_t s = (hipStream_t)stream;
    switch (tile_cfg) {
        case 0: return launch_cfg<128, 128, 2, 2>(args, ntiles, s);
        case 1: return launch_cfg<64, 128, 2, 2>(args, ntiles, s);
        case 2: return launch_cfg<32, 256, 1, 4>(args, ntiles, s);
    }
    ffc::set_error("ffc_conv_forward: unknown tile_cfg");
    return FFC_E_INVALID;
}

extern "C" int ffc_conv_pack(const ffc_conv_job* job, const float* const* seg_weight, const int* w_layout,
                             const int* kh, const int* kw, const float* const* seg_bias, float* A_out,
                             float* bias_out, void* stream) {
    FFC_CHECK_ARG(job && seg_weight && w_layout && kh && kw && A_out, "ffc_conv_pack: bad args");
    FFC_CHECK_ARG(job->nseg >= 1 && job->nseg <= FFC_MAX_SEG && job->nphase >= 1 && job->nphase <= FFC_MAX_PHASE,
                  "ffc_conv_pack: bad job");
    PackArgs a;
    a.job = *job;
    long long total = 0;
    for (int p = 0; p < job->nphase; ++p) total += (long long)job->Mpad * job->ph[p].Kpad;
    for (int s = 0; s < FFC_MAX_SEG; ++s) {
        const bool on = s < job->nseg;
        a.w[s] = on ? seg_weight[s] : nullptr;
        a.bias[s] = (on && seg_bias) ? seg_bias[s] : nullptr;
        a.layout[s] = on ? w_layout[s] : 0;
        a.kh[s] = on ? kh[s] : 1;
        a.kw[s] = on ? kw[s] : 1;
        if (on) FFC_CHECK_ARG(a.w[s] != nullptr, "ffc_conv_pack: null weight");
    }
    a.A = A_out;
    a.bias_out = bias_out;
    a.total = total;
    const long long work = total > job->M ? total : job->M;
    hipLaunchKernelGGL(conv_pack_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a);
    return ffc::launch_status("ffc_conv_pack");
}
