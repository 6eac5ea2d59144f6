// Direct (VALU) ConvTranspose2d k4 s2 p1 and Conv2d k3 s1 p1 for very few output channels
// (M <= 4) on gfx950.
//
// Conv2d k3 s1 p1 (conv3x3_smallm_kernel): the fgan128 generator's head conv7
// (FFC_BN_ACT(128, 3, 3, 0.5, 0, 1, 1, Tanh), fgan128_complete.py:484; local branch ffc.py:89-97)
// maps 2 x 64 channels to 3 at 128x128.  Same tiling and staging as the ConvT kernel below: a
// thread owns a 2x2 output block and reads its 4x4 input neighbourhood once per channel (16
// patch reads feed 36M FMAs); the chunk weights are staged as [channel][m][12] (9 taps, padded).
//
// The FFC-DCGAN generator's last layer (FFC_BN_ACT(ngf, nc, 4, 0.5, 0, 2, 1, Tanh),
// models/ffc_generator.py:28; local branch ffc_transpose.py:96-100) maps 2 x 32 channels
// to nc = 1 or 3 channels at 64x64.  An MFMA tile would be >90% padding, so this kernel
// computes it on the VALU.  Each thread owns a 2x2 block of input pixels (my, mx) and
// produces their 4x4 output pixels (2my+py, 2mx+px) for all M channels from the 4x4 input
// neighbourhood it reads once per channel:
//     py = 0: (ky=1, dy=0), (ky=3, dy=-1)      py = 1: (ky=0, dy=+1), (ky=2, dy=0)
// A workgroup covers a 32x32 input tile (+1 halo) with two halves of 256 threads that split the
// channel chunks (even / odd 8-channel chunks; two waves per SIMD) and add their partial sums
// in a fixed order at the end.  Each half's chunk of the tile and of the weights is staged in
// LDS by LDS-DMA (global_load_lds_dword, zero fill outside the image), double buffered; the
// weights of a channel are read as wave-uniform (broadcast) ds_read_b128 and reused by the
// thread's 4 pixels: per channel 16 patch reads + 4M broadcast reads feed 64M FMAs.
#include "ffc_internal.h"

namespace {

constexpr int CCH = 8;       // channels per chunk
constexpr int TT = 32;       // input tile (TT x TT), 16 x 16 threads x 2 x 2 pixels
constexpr int PP = TT + 2;   // patch side with halo
constexpr int PE = CCH * PP * PP;
constexpr int WE = CCH * 4 * 16;          // chunk weights (M <= 4)
constexpr int EBUF = ((PE + WE) + 255) & ~255;   // 4 buffers (2 halves x 2 stages) = 160 KiB
constexpr int SM_THREADS = 512;

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
    int nty, ntx;
    int act;
    float act_param;
};

template <int MM>
__global__ __launch_bounds__(SM_THREADS) void convt_smallm_kernel(SmallMArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int half = threadIdx.x >> 8, tid = threadIdx.x & 255, wave = tid >> 6;
    int bid = blockIdx.x;
    const int tx = bid % a.ntx;
    bid /= a.ntx;
    const int ty = bid % a.nty;
    const int b = bid / a.nty;
    const int y0 = ty * TT, x0 = tx * TT;
    const int qy = 2 * (tid >> 4), qx = 2 * (tid & 15);   // top-left of this thread's 2x2 pixels
    const int M = a.M;

    const int nch0 = (a.C[0] + CCH - 1) / CCH;
    const int nchunks = nch0 + (a.nseg > 1 ? (a.C[1] + CCH - 1) / CCH : 0);

    auto stage = [&](int ci, float* dst) {
        const int s = ci < nch0 ? 0 : 1;
        const int c0 = (s == 0 ? ci : ci - nch0) * CCH;
        const float* x = a.x[s];
        const float* w = a.w[s];
        const int C = a.C[s];
        const int wn = min(CCH, C - c0) * M * 16;
        for (int e = 0; e * 256 < PE + WE; ++e) {
            const int n = e * 256 + tid;
            const float* src = g_zero_sm;
            if (n < PE) {
                const int pc = n % PP, r = n / PP;
                const int pr = r % PP, ch = r / PP;
                const int iy = y0 - 1 + pr, ix = x0 - 1 + pc, c = c0 + ch;
                if (c < C && (unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW)
                    src = x + (((size_t)b * C + c) * a.IH + iy) * a.IW + ix;
            } else if (n - PE < wn) {
                src = w + (size_t)c0 * M * 16 + (n - PE);
            }
            __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(dst + e * 256 + wave * 64), 4, 0, 0);
        }
    };

    float acc[MM][4][4];   // [m][output row 0..3][output col 0..3] of the thread's 4x4 output block
#pragma unroll
    for (int m = 0; m < MM; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[m][i][j] = 0.0f;

    const int nsteps = (nchunks + 1) / 2;   // half h takes chunks 2k + h
    if (half < nchunks) stage(half, lds + half * EBUF);
    for (int k = 0; k < nsteps; ++k) {
        __syncthreads();
        const int ci = 2 * k + half;
        if (ci + 2 < nchunks) stage(ci + 2, lds + (((k + 1) & 1) * 2 + half) * EBUF);
        if (ci >= nchunks) continue;
        const float* cur = lds + ((k & 1) * 2 + half) * EBUF;
        const int s = ci < nch0 ? 0 : 1;
        const int c0 = (s == 0 ? ci : ci - nch0) * CCH;
        const int cn = min(CCH, a.C[s] - c0);
        for (int cc = 0; cc < cn; ++cc) {
            // 4x4 neighbourhood: input rows qy-1..qy+2, cols qx-1..qx+2 (patch has a +1 halo)
            float v[4][4];
            const float* p = cur + (cc * PP + qy) * PP + qx;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) v[i][j] = p[i * PP + j];
            const float* wl = cur + PE + cc * M * 16;
#pragma unroll
            for (int m = 0; m < MM; ++m) {
                if (m < M) {
                    float k[16];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float4 t = reinterpret_cast<const float4*>(wl + m * 16)[q];
                        k[4 * q] = t.x; k[4 * q + 1] = t.y; k[4 * q + 2] = t.z; k[4 * q + 3] = t.w;
                    }
                    // input pixel (qy+aa, qx+cb); output row 2aa+py, col 2cb+px
#pragma unroll
                    for (int aa = 0; aa < 2; ++aa)
#pragma unroll
                        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
                            for (int py = 0; py < 2; ++py)
#pragma unroll
                                for (int px = 0; px < 2; ++px) {
                                    float s2 = acc[m][2 * aa + py][2 * cb + px];
#pragma unroll
                                    for (int ta = 0; ta < 2; ++ta)
#pragma unroll
                                        for (int tb = 0; tb < 2; ++tb) {
                                            const int ky = py == 0 ? (ta == 0 ? 1 : 3) : (ta == 0 ? 0 : 2);
                                            const int dy = py == 0 ? (ta == 0 ? 0 : -1) : (ta == 0 ? 1 : 0);
                                            const int kx = px == 0 ? (tb == 0 ? 1 : 3) : (tb == 0 ? 0 : 2);
                                            const int dx = px == 0 ? (tb == 0 ? 0 : -1) : (tb == 0 ? 1 : 0);
                                            s2 = fmaf(v[aa + dy + 1][cb + dx + 1], k[ky * 4 + kx], s2);
                                        }
                                    acc[m][2 * aa + py][2 * cb + px] = s2;
                                }
                }
            }
        }
    }
    // fixed-order combine of the two halves' partial sums (half 1 -> LDS -> half 0 adds)
    __syncthreads();
    float* part = lds;   // 256 threads x MM x 16 (the stage buffers are free now)
    if (half == 1) {
#pragma unroll
        for (int m = 0; m < MM; ++m)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) part[((m * 4 + i) * 4 + j) * 256 + tid] = acc[m][i][j];
    }
    __syncthreads();
    if (half == 1) return;
#pragma unroll
    for (int m = 0; m < MM; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[m][i][j] += part[((m * 4 + i) * 4 + j) * 256 + tid];
    const int OH = 2 * a.IH, OW = 2 * a.IW;
    const int oy0 = 2 * (y0 + qy), ox0 = 2 * (x0 + qx);
    const bool xin = x0 + qx + 1 < a.IW;   // both input columns in range
    auto store = [&](auto actf) {
#pragma unroll
        for (int m = 0; m < MM; ++m) {
            if (m >= M) break;
            const float bv = a.bias ? a.bias[m] : 0.0f;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int oy = oy0 + i;
                if (oy >= OH) continue;
                float* row = a.out + (((size_t)b * M + m) * OH + oy) * OW + ox0;
                if (xin) {
                    *reinterpret_cast<float4*>(row) = make_float4(actf(acc[m][i][0] + bv), actf(acc[m][i][1] + bv),
                                                                  actf(acc[m][i][2] + bv), actf(acc[m][i][3] + bv));
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (ox0 + j < OW) row[j] = actf(acc[m][i][j] + bv);
                }
            }
        }
    };
    const float ap = a.act_param;
    switch (a.act) {
        case FFC_ACT_RELU: store([](float v) { return fmaxf(v, 0.0f); }); break;
        case FFC_ACT_LEAKY_RELU: store([ap](float v) { return v > 0.0f ? v : v * ap; }); break;
        case FFC_ACT_TANH: store([](float v) { return tanhf(v); }); break;
        case FFC_ACT_SIGMOID: store([](float v) { return 1.0f / (1.0f + expf(-v)); }); break;
        case FFC_ACT_GELU: store([](float v) { return 0.5f * v * (1.0f + erff(v * 0.70710678118654752f)); }); break;
        default: store([](float v) { return v; }); break;
    }
}


// ---- Conv2d k3 s1 p1, M <= 4: 64x64 output tile per workgroup, 4x4 outputs per thread.
// The input patch row covers ix = x0-4 .. x0+67 (72 floats = 18 aligned float4 groups; W % 4 == 0,
// so a group is wholly inside or outside the image).  The two halves of the workgroup take
// alternate channels; each stages one channel per step through registers: the global loads of
// channel k+1 are issued before channel k's FMAs and written to the other LDS buffer after them
// (an LDS-DMA pipeline would not overlap: the compiler waits for every outstanding LDS-DMA before
// any LDS read).  All weights are staged once, as [channel][m][12] (9 taps, padded).
// Per channel a thread reads its 6x6 neighbourhood as 6 x (b32 + b128 + b32) and 3 x 3 broadcast
// b128 of weights: 18 + 3M LDS reads feed 144M FMAs.
constexpr int T3 = 64;                      // output tile side
constexpr int R3 = T3 + 2;                  // patch rows (halo 1)
constexpr int S3 = T3 + 8;                  // patch row: 18 float4 groups
constexpr int G3 = R3 * (S3 / 4);           // float4 groups per channel
constexpr int GT3 = (G3 + 255) / 256;       // groups per thread
constexpr int PB3 = G3 * 4;                 // floats per patch buffer
constexpr int CMAX3 = 256;                  // channels (both segments) whose weights fit the LDS slot

template <int MM>
__global__ __launch_bounds__(SM_THREADS) void conv3x3_smallm_kernel(SmallMArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int half = threadIdx.x >> 8, tid = threadIdx.x & 255;
    int bid = blockIdx.x;
    const int tx = bid % a.ntx;
    bid /= a.ntx;
    const int ty = bid % a.nty;
    const int b = bid / a.nty;
    const int y0 = ty * T3, x0 = tx * T3;
    const int qy = 4 * (tid >> 4), qx = 4 * (tid & 15);   // this thread's 4x4 outputs (tile coords)
    const int M = a.M;
    const int nchunks = a.C[0] + (a.nseg > 1 ? a.C[1] : 0);   // one channel per chunk
    float* wl_all = lds;                                      // [nchunks][4][12]
    float* pbuf = lds + CMAX3 * 48;                           // [2 buffers][2 halves][PB3]

    for (int q0 = 0; q0 < nchunks * 48; q0 += 8 * SM_THREADS) {   // 8 loads in flight per thread
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int q = q0 + u * SM_THREADS + threadIdx.x;
            const int ci = q / 48, m = (q / 12) & 3, t = q % 12;
            const int s = ci < a.C[0] ? 0 : 1;
            const int c = s == 0 ? ci : ci - a.C[0];
            v[u] = (q < nchunks * 48 && t < 9 && m < M) ? a.w[s][((size_t)m * a.C[s] + c) * 9 + t] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int q = q0 + u * SM_THREADS + threadIdx.x;
            if (q < nchunks * 48) wl_all[q] = v[u];
        }
    }

    auto load = [&](int ci, float4 (&r)[GT3]) {
        const int s = ci < a.C[0] ? 0 : 1;
        const int c = s == 0 ? ci : ci - a.C[0];
        const float* x = a.x[s] + ((size_t)b * a.C[s] + c) * a.IH * a.IW;
#pragma unroll
        for (int j = 0; j < GT3; ++j) {
            const int n = j * 256 + tid;
            const int g = n % (S3 / 4), pr = n / (S3 / 4);
            const int iy = y0 - 1 + pr, ix = x0 - 4 + 4 * g;
            r[j] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (n < G3 && (unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW)
                r[j] = *reinterpret_cast<const float4*>(x + (size_t)iy * a.IW + ix);
        }
    };
    auto put = [&](float* dst, const float4 (&r)[GT3]) {
#pragma unroll
        for (int j = 0; j < GT3; ++j) {
            const int n = j * 256 + tid;
            if (n < G3) reinterpret_cast<float4*>(dst)[n] = r[j];
        }
    };
    auto buf = [&](int k) { return pbuf + ((k & 1) * 2 + half) * PB3; };

    float acc[MM][4][4];
#pragma unroll
    for (int m = 0; m < MM; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[m][i][j] = 0.0f;

    const int nsteps = (nchunks + 1) / 2;   // half h takes chunks 2k + h (its k-th channel)
    auto compute = [&](int k) {
        const int ci = 2 * k + half;
        if (ci >= nchunks) return;
        const float* cur = buf(k);
        float v[6][6];   // input rows qy-1..qy+4, cols qx-1..qx+4 = patch rows qy..qy+5, cols qx+3..qx+8
        const float* p = cur + qy * S3 + qx + 3;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const float4 l4 = *reinterpret_cast<const float4*>(p + i * S3 + 1);
            v[i][0] = p[i * S3];
            v[i][1] = l4.x; v[i][2] = l4.y; v[i][3] = l4.z; v[i][4] = l4.w;
            v[i][5] = p[i * S3 + 5];
        }
        const float* wl = wl_all + ci * 48;
#pragma unroll
        for (int m = 0; m < MM; ++m) {
            float k9[12];
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const float4 t = reinterpret_cast<const float4*>(wl + m * 12)[q];
                k9[4 * q] = t.x; k9[4 * q + 1] = t.y; k9[4 * q + 2] = t.z; k9[4 * q + 3] = t.w;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    float s2 = acc[m][i][j];
#pragma unroll
                    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                        for (int kx = 0; kx < 3; ++kx) s2 = fmaf(v[i + ky][j + kx], k9[ky * 3 + kx], s2);
                    acc[m][i][j] = s2;
                }
        }
    };
    // one channel of prefetch in registers: channel k+1's loads are in flight under channel k's FMAs
    // (a second register set measured slower: 196 VGPRs, same occupancy)
    float4 r[GT3];
    if (half < nchunks) {
        load(half, r);
        put(buf(0), r);
    }
    __syncthreads();
    for (int k = 0; k < nsteps; ++k) {
        const int cn = 2 * (k + 1) + half;
        if (cn < nchunks) load(cn, r);
        compute(k);
        if (cn < nchunks) put(buf(k + 1), r);
        __syncthreads();
    }
    // fixed-order combine of the two halves' partial sums (half 1 -> LDS -> half 0 adds)
    float* part = pbuf;   // 256 threads x MM x 16 floats <= 4 * PB3
    if (half == 1) {
#pragma unroll
        for (int m = 0; m < MM; ++m)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) part[((m * 4 + i) * 4 + j) * 256 + tid] = acc[m][i][j];
    }
    __syncthreads();
    if (half == 1) return;
#pragma unroll
    for (int m = 0; m < MM; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[m][i][j] += part[((m * 4 + i) * 4 + j) * 256 + tid];
    const int oy0 = y0 + qy, ox0 = x0 + qx;
    const bool xin = ox0 + 3 < a.IW;
    auto store = [&](auto actf) {
#pragma unroll
        for (int m = 0; m < MM; ++m) {
            if (m >= M) break;
            const float bv = a.bias ? a.bias[m] : 0.0f;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int oy = oy0 + i;
                if (oy >= a.IH) continue;
                float* row = a.out + (((size_t)b * M + m) * a.IH + oy) * a.IW + ox0;
                if (xin) {
                    *reinterpret_cast<float4*>(row) = make_float4(actf(acc[m][i][0] + bv), actf(acc[m][i][1] + bv),
                                                                  actf(acc[m][i][2] + bv), actf(acc[m][i][3] + bv));
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (ox0 + j < a.IW) row[j] = actf(acc[m][i][j] + bv);
                }
            }
        }
    };
    const float ap = a.act_param;
    switch (a.act) {
        case FFC_ACT_RELU: store([](float v) { return fmaxf(v, 0.0f); }); break;
        case FFC_ACT_LEAKY_RELU: store([ap](float v) { return v > 0.0f ? v : v * ap; }); break;
        case FFC_ACT_TANH: store([](float v) { return tanhf(v); }); break;
        case FFC_ACT_SIGMOID: store([](float v) { return 1.0f / (1.0f + expf(-v)); }); break;
        case FFC_ACT_GELU: store([](float v) { return 0.5f * v * (1.0f + erff(v * 0.70710678118654752f)); }); break;
        default: store([](float v) { return v; }); break;
    }
}

}  // namespace

extern "C" int ffc_convt_k4s2_smallm(const float* x0, int C0, const float* w0, const float* x1, int C1,
                                     const float* w1, const float* bias, int B, int IH, int IW, int M,
                                     float* out, int act, float act_param, void* stream) {
    FFC_CHECK_ARG(x0 && w0 && out && B > 0 && IH > 0 && IW > 0 && C0 > 0, "ffc_convt_k4s2_smallm: bad args");
    FFC_CHECK_ARG(M >= 1 && M <= 4, "ffc_convt_k4s2_smallm: 1 <= M <= 4");
    FFC_CHECK_ARG(!x1 || (w1 && C1 > 0), "ffc_convt_k4s2_smallm: second segment");
    FFC_CHECK_ARG((reinterpret_cast<uintptr_t>(out) & 15) == 0, "ffc_convt_k4s2_smallm: output not 16-B aligned");
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
    a.nty = (IH + TT - 1) / TT;
    a.ntx = (IW + TT - 1) / TT;
    a.act = act;
    a.act_param = act_param;
    const size_t lds = 4 * (size_t)EBUF * sizeof(float);
    const unsigned grid = (unsigned)B * a.nty * a.ntx;
    auto k = convt_smallm_kernel<4>;
    static bool raised = false;
    if (!raised) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024) != hipSuccess) {
            ffc::set_error("ffc_convt_k4s2_smallm: hipFuncSetAttribute failed");
            return FFC_E_LAUNCH;
        }
        raised = true;
    }
    hipLaunchKernelGGL(k, dim3(grid), dim3(SM_THREADS), lds, (hipStream_t)stream, a);
    return ffc::launch_status("ffc_convt_k4s2_smallm");
}

extern "C" int ffc_conv3x3_smallm(const float* x0, int C0, const float* w0, const float* x1, int C1,
                                  const float* w1, const float* bias, int B, int H, int W, int M, float* out,
                                  int act, float act_param, void* stream) {
    FFC_CHECK_ARG(x0 && w0 && out && B > 0 && H > 0 && W > 0 && C0 > 0, "ffc_conv3x3_smallm: bad args");
    FFC_CHECK_ARG(M >= 1 && M <= 4, "ffc_conv3x3_smallm: 1 <= M <= 4");
    FFC_CHECK_ARG(!x1 || (w1 && C1 > 0), "ffc_conv3x3_smallm: second segment");
    FFC_CHECK_ARG((reinterpret_cast<uintptr_t>(out) & 15) == 0 && W % 4 == 0,
                  "ffc_conv3x3_smallm: output not 16-B aligned or W % 4 != 0");
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
    a.IH = H;
    a.IW = W;
    a.M = M;
    a.nty = (H + T3 - 1) / T3;
    a.ntx = (W + T3 - 1) / T3;
    a.act = act;
    a.act_param = act_param;
    FFC_CHECK_ARG(C0 + (x1 ? C1 : 0) <= CMAX3, "ffc_conv3x3_smallm: at most 256 input channels");
    const size_t lds = (CMAX3 * 48 + 4 * (size_t)PB3) * sizeof(float);
    const unsigned grid = (unsigned)B * a.nty * a.ntx;
    // M is a template parameter: no runtime m < M branches in the FMA body
    auto k = M == 1 ? conv3x3_smallm_kernel<1> : M == 2 ? conv3x3_smallm_kernel<2>
           : M == 3 ? conv3x3_smallm_kernel<3> : conv3x3_smallm_kernel<4>;
    static bool raised[5] = {false, false, false, false, false};
    if (!raised[M]) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024) != hipSuccess) {
            ffc::set_error("ffc_conv3x3_smallm: hipFuncSetAttribute failed");
            return FFC_E_LAUNCH;
        }
        raised[M] = true;
    }
    hipLaunchKernelGGL(k, dim3(grid), dim3(SM_THREADS), lds, (hipStream_t)stream, a);
    return ffc::launch_status("ffc_conv3x3_smallm");
}
