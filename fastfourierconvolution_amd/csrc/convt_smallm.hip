// Direct (VALU) ConvTranspose2d k4 s2 p1 for very few output channels (M <= 4) on gfx950.
//
// The FFC-DCGAN generator's last layer (FFC_BN_ACT(ngf, nc, 4, 0.5, 0, 2, 1, Tanh),
// models/ffc_generator.py:28; local branch ffc_transpose.py:96-100) maps 2 x 32 channels
// to nc = 1 or 3 channels at 64x64.  An MFMA tile would be >90% padding, so this kernel
// computes it on the VALU: each thread owns one input pixel (my, mx) and produces the 2x2
// output pixels (2my+py, 2mx+px) of all M channels from the 3x3 input neighbourhood:
//     py = 0: (ky=1, dy=0), (ky=3, dy=-1)      py = 1: (ky=0, dy=+1), (ky=2, dy=0)
// 16-channel input patches (tile + 1-pixel halo) are staged in LDS by LDS-DMA
// (global_load_lds_dword, zero fill outside the image), double buffered; weights are
// wave-uniform and come through the scalar cache.  Per channel: 9 LDS reads, 16*M FMAs.
#include "ffc_internal.h"

namespace {

constexpr int CCH = 16;
__device__ float g_zero_sm[64];
typedef __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

struct SmallMArgs {
    const float* x[2];
    const float* w[2];   // ConvTranspose2d weights (C_s, M, 4, 4)
    int C[2];
    int nseg;
    const float* bias;
    float* out;          // (B, M, 2IH, 2IW)
    int B, IH, IW, M;
    int TRw, TCw, nty, ntx;
    int act;
    float act_param;
};

template <int MM>
__global__ __launch_bounds__(256) void convt_smallm_kernel(SmallMArgs a, const float* __restrict__ wseg0,
                                                           const float* __restrict__ wseg1) {
    extern __shared__ __attribute__((aligned(16))) float patch[];
    const int tid = threadIdx.x, wave = tid >> 6;
    const int TRw = a.TRw, TCw = a.TCw;
    const int PR = TRw + 2, PC = TCw + 2, PE = CCH * PR * PC;
    const int ebuf = (PE + 255) & ~255;
    int bid = blockIdx.x;
    const int tx = bid % a.ntx;
    bid /= a.ntx;
    const int ty = bid % a.nty;
    const int b = bid / a.nty;
    const int y0 = ty * TRw, x0 = tx * TCw;
    const int qy = tid / TCw, qx = tid - qy * TCw;
    const int my = y0 + qy, mx = x0 + qx;
    const bool valid = qy < TRw && my < a.IH && mx < a.IW;

    const int nch0 = (a.C[0] + CCH - 1) / CCH;
    const int nchunks = nch0 + (a.nseg > 1 ? (a.C[1] + CCH - 1) / CCH : 0);

    auto stage = [&](int ci, float* dst) {
        const int s = ci < nch0 ? 0 : 1;
        const int c0 = (s == 0 ? ci : ci - nch0) * CCH;
        const float* x = a.x[s];
        const int C = a.C[s];
        for (int e = 0; e * 256 < PE; ++e) {
            const int n = e * 256 + tid;
            const int pc = n % PC, r = n / PC;
            const int pr = r % PR, ch = r / PR;
            const int iy = y0 - 1 + pr, ix = x0 - 1 + pc, c = c0 + ch;
            const bool ok = n < PE && c < C && (unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW;
            const float* src = ok ? x + (((size_t)b * C + c) * a.IH + iy) * a.IW + ix : g_zero_sm;
            __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(dst + e * 256 + wave * 64), 4, 0, 0);
        }
    };

    float acc[MM][4];
#pragma unroll
    for (int m = 0; m < MM; ++m)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[m][q] = 0.0f;

    stage(0, patch);
    for (int ci = 0; ci < nchunks; ++ci) {
        __syncthreads();
        if (ci + 1 < nchunks) stage(ci + 1, patch + ((ci + 1) & 1) * ebuf);
        const float* cur = patch + (ci & 1) * ebuf;
        const int s = ci < nch0 ? 0 : 1;
        const int c0 = (s == 0 ? ci : ci - nch0) * CCH;
        const int cn = min(CCH, a.C[s] - c0);
        const float* __restrict__ w = s == 0 ? wseg0 : wseg1;
        for (int cc = 0; cc < cn; ++cc) {
            const float* p = cur + (cc * PR + qy + 1) * PC + qx + 1;
            float v[3][3];
#pragma unroll
            for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
                for (int dx = -1; dx <= 1; ++dx) v[dy + 1][dx + 1] = p[dy * PC + dx];
            // wave-uniform weight address in SGPRs -> scalar (s_load) weight reads
            const float* wc = w + __builtin_amdgcn_readfirstlane((c0 + cc) * a.M * 16);
#pragma unroll
            for (int m = 0; m < MM; ++m) {
                if (m < a.M) {
                    float k[16];
#pragma unroll
                    for (int i = 0; i < 16; ++i) k[i] = wc[m * 16 + i];
                    // out(2my+py, 2mx+px): rows (ky, dy) = py0: (1,0),(3,-1)  py1: (0,+1),(2,0)
#pragma unroll
                    for (int py = 0; py < 2; ++py)
#pragma unroll
                        for (int px = 0; px < 2; ++px) {
                            float s2 = acc[m][py * 2 + px];
#pragma unroll
                            for (int ta = 0; ta < 2; ++ta)
#pragma unroll
                                for (int tb = 0; tb < 2; ++tb) {
                                    const int ky = py == 0 ? (ta == 0 ? 1 : 3) : (ta == 0 ? 0 : 2);
                                    const int dy = py == 0 ? (ta == 0 ? 0 : -1) : (ta == 0 ? 1 : 0);
                                    const int kx = px == 0 ? (tb == 0 ? 1 : 3) : (tb == 0 ? 0 : 2);
                                    const int dx = px == 0 ? (tb == 0 ? 0 : -1) : (tb == 0 ? 1 : 0);
                                    s2 = fmaf(v[dy + 1][dx + 1], k[ky * 4 + kx], s2);
                                }
                            acc[m][py * 2 + px] = s2;
                        }
                }
            }
        }
    }
    if (!valid) return;
    const int OH = 2 * a.IH, OW = 2 * a.IW;
#pragma unroll
    for (int m = 0; m < MM; ++m) {
        if (m >= a.M) break;
        const float bv = a.bias ? a.bias[m] : 0.0f;
#pragma unroll
        for (int py = 0; py < 2; ++py) {
            float2 r;
            r.x = ffc::apply_act(acc[m][py * 2 + 0] + bv, a.act, a.act_param);
            r.y = ffc::apply_act(acc[m][py * 2 + 1] + bv, a.act, a.act_param);
            *reinterpret_cast<float2*>(a.out + (((size_t)b * a.M + m) * OH + 2 * my + py) * OW + 2 * mx) = r;
        }
    }
}

}  // namespace

extern "C" int ffc_convt_k4s2_smallm(const float* x0, int C0, const float* w0, const float* x1, int C1,
                                     const float* w1, const float* bias, int B, int IH, int IW, int M,
                                     float* out, int act, float act_param, void* stream) {
    FFC_CHECK_ARG(x0 && w0 && out && B > 0 && IH > 0 && IW > 0 && C0 > 0, "ffc_convt_k4s2_smallm: bad args");
    FFC_CHECK_ARG(M >= 1 && M <= 4, "ffc_convt_k4s2_smallm: 1 <= M <= 4");
    FFC_CHECK_ARG(!x1 || (w1 && C1 > 0), "ffc_convt_k4s2_smallm: second segment");
    SmallMArgs a;
    a.x[0] = x0;
    a.w[0] = w0;
    a.C[0] = C0;
    a.x[1] = x1;
    a.w[1] = w1;
    a.C[1] = x1 ? C1 : 0;
    a.nseg = x1 ? 2 : 1;
    a.bias = bias;
    a.out = out;
    a.B = B;
    a.IH = IH;
    a.IW = IW;
    a.M = M;
    a.TCw = IW >= 32 ? 32 : IW;
    a.TRw = 256 / a.TCw;
    a.nty = (IH + a.TRw - 1) / a.TRw;
    a.ntx = (IW + a.TCw - 1) / a.TCw;
    a.act = act;
    a.act_param = act_param;
    const int PE = CCH * (a.TRw + 2) * (a.TCw + 2);
    const size_t lds = 2 * (size_t)((PE + 255) & ~255) * sizeof(float);
    FFC_CHECK_ARG(lds <= 64 * 1024, "ffc_convt_k4s2_smallm: tile too large");
    const unsigned grid = (unsigned)B * a.nty * a.ntx;
    hipLaunchKernelGGL(convt_smallm_kernel<4>, dim3(grid), dim3(256), lds, (hipStream_t)stream, a, w0,
                       x1 ? w1 : w0);
    return ffc::launch_status("ffc_convt_k4s2_smallm");
}
