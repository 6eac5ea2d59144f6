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
// to nc = 1 or 3 channels at 64x64 (convt_smallm_kernel).  An MFMA tile would be >90% padding,
// so it runs on the VALU.  Each thread owns a 2x2 block of input pixels (my, mx) and produces
// their 4x4 output pixels (2my+py, 2mx+px) for all M channels from the 4x4 input neighbourhood
// it reads once per channel:
//     py = 0: (ky=1, dy=0), (ky=3, dy=-1)      py = 1: (ky=0, dy=+1), (ky=2, dy=0)
// A workgroup covers a 32x16 input tile (+1 halo) with four quarters of 128 threads that take
// alternate channels and add their partial sums in a fixed order at the end; two workgroups per
// CU.  The weights are packed once as [channel][tap][m 0..3] and read per channel by scalar loads,
// so the FMAs run as v_pk_fma_f32 on output-channel pairs (one input value against two channels'
// SGPR weights).  Each quarter stages
// its next channel's patch through registers (float4 loads issued before the current channel's
// FMAs, written to the other LDS buffer after them).
#include "ffc_internal.h"

#include <algorithm>
#include <cstdlib>

namespace {

constexpr int SM_THREADS = 512;   // conv3x3_smallm_kernel: two halves of 256

// exact GELU x * Phi(x) (nn.GELU(approximate='none')) with erf from Abramowitz & Stegun 7.1.26
// (|erf error| <= 1.5e-7, so |GELU error| <= 0.75e-7 |x|): one reciprocal, one exp and five FMAs on
// a single branch-free path
__device__ __forceinline__ float gelu_as(float v) {
    const float z = fabsf(v) * 0.70710678118654752f;
    const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
    float q = fmaf(t, 1.061405429f, -1.453152027f);
    q = fmaf(q, t, 1.421413741f);
    q = fmaf(q, t, -0.284496736f);
    q = fmaf(q, t, 0.254829592f);
    const float e = q * t * __expf(-z * z);    // erfc(z)
    const float h = 0.5f * v * e;
    return v >= 0.0f ? v - h : h;
}

typedef float f2 __attribute__((ext_vector_type(2)));

// gelu_as on two values at once: the polynomial, the exp argument and the products run as packed
// v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 (rcp and exp have no packed form), ~40 % fewer issue
// slots than two gelu_as -- the head conv's deferred transform is VALU-bound.  Same expression per
// element as gelu_as (results bit-identical up to fma contraction of the exp argument).
__device__ __forceinline__ f2 gelu_as2(f2 v) {
    const f2 z = f2{fabsf(v.x), fabsf(v.y)} * 0.70710678118654752f;
    const f2 d = z * 0.3275911f + 1.0f;
    const f2 t = f2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
    f2 q = t * 1.061405429f - 1.453152027f;
    q = q * t + 1.421413741f;
    q = q * t - 0.284496736f;
    q = q * t + 0.254829592f;
    const f2 zz = -(z * z);
    const f2 e = q * t * f2{__expf(zz.x), __expf(zz.y)};   // erfc(z)
    const f2 h = 0.5f * v * e;
    const f2 r = v - h;
    return f2{v.x >= 0.0f ? r.x : h.x, v.y >= 0.0f ? r.y : h.y};
}

struct SmallMArgs {
    const float* x[2];
    const float* w[2];   // Conv2d (M, C_s, 3, 3) weights (conv3x3_smallm_kernel)
    const float* wpack;  // ConvTranspose2d weights packed [C0 + C1][16][4] (convt_smallm_kernel)
    int C[2];
    int nseg;
    const float* bias;
    float* out;
    int B, IH, IW, M;
    int nty, ntx;
    int comb;            // convt_smallm_kernel quarter combine: 0 serial, 1 all quarters at once (8 x 1 wave), 2 one barrier into quarter 0
    int act;
    float act_param;
    ffc_in_tf tf[2];     // conv3x3_smallm_kernel<MM, true>: deferred BN + act (+ noise) of segment s
};

// ---- ConvTranspose2d k4 s2 p1, M <= 4: 32x32 input tile (64x64 outputs) per workgroup.
constexpr int CT_TT = 32;                    // input tile columns; a thread owns 2x2 input pixels
#ifndef FFC_CT_TR
#define FFC_CT_TR 16
#endif
#ifndef FFC_CT_CPQ
#define FFC_CT_CPQ 2
#endif
#ifndef FFC_CT_ONECOMB
#define FFC_CT_ONECOMB 1   // 0: the serial quarter combine everywhere (A/B)
#endif
constexpr int CT_TR = FFC_CT_TR;             // input tile rows
constexpr int CT_QT = (CT_TT / 2) * (CT_TR / 2);   // threads per channel quarter
constexpr int CT_PR = CT_TR + 2;             // patch rows: iy = y0-1 .. y0+TR
constexpr int CT_PS = CT_TT + 8;             // patch row: ix = x0-4 .. x0+35 (10 aligned float4 groups)
constexpr int CT_G = CT_PR * (CT_PS / 4);    // float4 groups per channel
constexpr int CT_CPQ = FFC_CT_CPQ;           // channels per quarter per step
constexpr int CT_GT = (CT_CPQ * CT_G + CT_QT - 1) / CT_QT;   // groups per thread per step
constexpr int CT_PB = CT_PR * CT_PS;         // floats per channel patch
constexpr int CT_NQ = 4;                     // channel quarters
constexpr int CT_THREADS = CT_QT * CT_NQ;
constexpr int CT_CMAX = 256;                 // channels (both segments)

// MM output channels: pairs (m, m+1) run as v_pk_fma_f32, one input value against the two
// channels' weights (packed layout [channel][tap][m 0..3]); an odd last channel is scalar.
// TR_ / NQ_: input tile rows and channel quarters.  The default 16 x 4 (512 threads) tiles large
// batches; 8 x 8 (same 512 threads, half the rows, the channels split 8 ways) doubles the workgroups
// when the grid would leave CUs idle (the small per-rank batches of strong scaling).
template <int MM, bool VEC, int TR_ = CT_TR, int NQ_ = CT_NQ>   // VEC: IW % 4 == 0 (whole float4 groups)
__global__ __launch_bounds__((CT_TT / 2) * (TR_ / 2) * NQ_) __attribute__((amdgpu_waves_per_eu(4))) void convt_smallm_kernel(SmallMArgs a) {
    constexpr int CT_TR = TR_, CT_NQ = NQ_;
    constexpr int CT_QT = (CT_TT / 2) * (CT_TR / 2);
    constexpr int CT_PR = CT_TR + 2;
    constexpr int CT_G = CT_PR * (CT_PS / 4);
    constexpr int CT_GT = (CT_CPQ * CT_G + CT_QT - 1) / CT_QT;
    constexpr int CT_PB = CT_PR * CT_PS;
    constexpr int CT_THREADS = CT_QT * CT_NQ;
    // the partial-sum combine area reuses the patch double buffer
    static_assert(CT_QT % 64 == 0 && CT_QT * 16 * 4 <= 2 * CT_NQ * CT_CPQ * CT_PB, "quarters of whole waves; combine area fits");
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int q = __builtin_amdgcn_readfirstlane(threadIdx.x / CT_QT), tid = threadIdx.x % CT_QT;
    int bid = blockIdx.x;
    const int tx = bid % a.ntx;
    bid /= a.ntx;
    const int ty = bid % a.nty;
    const int b = bid / a.nty;
    const int y0 = ty * CT_TR, x0 = tx * CT_TT;
    const int qy = 2 * (tid >> 4), qx = 2 * (tid & 15);   // top-left of this thread's 2x2 input pixels
    const int M = a.M, C0 = a.C[0];
    const int Ct = C0 + (a.nseg > 1 ? a.C[1] : 0);
    // one base plus a per-lane offset: a lane-varying select between a.x[0] and a.x[1] is folded
    // into a per-lane load of the selected kernel argument
    const float* xs0 = a.x[0];
    const long long xd1 = a.nseg > 1 ? (long long)(a.x[1] - a.x[0]) : 0;   // segment 1 base - segment 0 base
    float* pbuf = lds;   // [2 stages][NQ][CPQ][PB]
    // packed weights [Ct][16 taps][4 m] (ffc_convt_smallm_pack), read per channel by scalar loads
    typedef float fx4 __attribute__((ext_vector_type(4)));

    // step k of quarter q: channels CPQ (NQ k + q) + {0 .. CPQ-1}
    auto load = [&](int k, float4 (&r)[CT_GT]) {
#pragma unroll
        for (int j = 0; j < CT_GT; ++j) {
            const int n = j * CT_QT + tid;
            const int cl = n / CT_G, nn = n - cl * CT_G;
            const int ci = CT_CPQ * (CT_NQ * k + q) + cl;
            const int g = nn % (CT_PS / 4), pr = nn / (CT_PS / 4);
            const int iy = y0 - 1 + pr, ix = x0 - 4 + 4 * g;
            const bool rok = n < CT_CPQ * CT_G && ci < Ct && (unsigned)iy < (unsigned)a.IH;
            const size_t ihw = (size_t)a.IH * a.IW;
            const float* x = xs0 + (ci < C0 ? (long long)((size_t)b * C0 + ci) * ihw
                                            : xd1 + (long long)((size_t)b * a.C[1] + (ci - C0)) * ihw);
            const float* row = x + (size_t)iy * a.IW;
            if (VEC) {
                // unconditional load at a clamped address, then a select: a load under a branch
                // is waited for before the next one issues
                const bool ok = rok && (unsigned)ix < (unsigned)a.IW;
                const float4 v = *reinterpret_cast<const float4*>(ok ? row + ix : xs0);
                r[j] = ok ? v : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            } else {
                r[j] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                if (!rok) continue;
                if ((unsigned)ix < (unsigned)a.IW) r[j].x = row[ix];
                if ((unsigned)(ix + 1) < (unsigned)a.IW) r[j].y = row[ix + 1];
                if ((unsigned)(ix + 2) < (unsigned)a.IW) r[j].z = row[ix + 2];
                if ((unsigned)(ix + 3) < (unsigned)a.IW) r[j].w = row[ix + 3];
            }
        }
    };
    auto put = [&](float* dst, const float4 (&r)[CT_GT]) {
#pragma unroll
        for (int j = 0; j < CT_GT; ++j) {
            const int n = j * CT_QT + tid;
            if (n < CT_CPQ * CT_G) reinterpret_cast<float4*>(dst)[n] = r[j];
        }
    };
    auto buf = [&](int k) { return pbuf + ((k & 1) * CT_NQ + q) * CT_CPQ * CT_PB; };

    constexpr int NPR = MM / 2, NSG = MM % 2;
    // [output row * 4 + output col] of the thread's 4x4 block: channel pairs, odd last channel
    f2 accp[16][NPR > 0 ? NPR : 1];
    float accs[16][NSG > 0 ? NSG : 1];
#pragma unroll
    for (int o = 0; o < 16; ++o) {
#pragma unroll
        for (int mp = 0; mp < NPR; ++mp) accp[o][mp] = f2{0.0f, 0.0f};
        if (NSG) accs[o][0] = 0.0f;
    }
    auto get = [&](int o, int m) -> float {
        if (m < 2 * NPR) return (m & 1) ? accp[o][m >> 1].y : accp[o][m >> 1].x;
        return accs[o][0];
    };
    auto add = [&](int o, int m, float v) {
        if (m < 2 * NPR) {
            if (m & 1) accp[o][m >> 1].y += v;
            else accp[o][m >> 1].x += v;
        } else {
            accs[o][0] += v;
        }
    };

    // out[oy] += x[iy] w[ky] with oy = 2 iy - 1 + ky: output row 2(qy+aa)+py takes input row
    // qy+aa+dy through ky = py + 1 - 2 dy (same for columns)
    auto compute = [&](int k, int cl) {
        const int ci = CT_CPQ * (CT_NQ * k + q) + cl;
        if (ci >= Ct) return;
        const float* p = buf(k) + cl * CT_PB + qy * CT_PS + qx + 3;   // input row qy-1, col qx-1
        float v[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const f2 mid = *reinterpret_cast<const f2*>(p + i * CT_PS + 1);
            v[i][0] = p[i * CT_PS];
            v[i][1] = mid.x;
            v[i][2] = mid.y;
            v[i][3] = p[i * CT_PS + 3];
        }
        // the channel's weights are wave-uniform: scalar loads (s_load_dwordx16) into SGPRs, read by
        // the FMAs directly.  Broadcast LDS reads of them (r03) returned 64 lanes x 16 B per tap and
        // bounded the kernel on LDS bandwidth (45 -> 39 us at gen64 B = 256, profiles/r04/z)
        const fx4* wg = reinterpret_cast<const fx4*>(a.wpack) + ci * 16;
#pragma unroll
        for (int ky = 0; ky < 4; ++ky) {
            const int py = (ky & 1) ? 0 : 1, dy = ky == 0 ? 1 : (ky == 3 ? -1 : 0);
#pragma unroll
            for (int kx = 0; kx < 4; ++kx) {
                const fx4 wk = wg[ky * 4 + kx];
                const int px = (kx & 1) ? 0 : 1, dx = kx == 0 ? 1 : (kx == 3 ? -1 : 0);
#pragma unroll
                for (int aa = 0; aa < 2; ++aa)
#pragma unroll
                    for (int cb = 0; cb < 2; ++cb) {
                        const float xv = v[aa + dy + 1][cb + dx + 1];
                        const int o = (2 * aa + py) * 4 + 2 * cb + px;
                        const f2 xx = f2{xv, xv};
                        if (NPR > 0) accp[o][0] = __builtin_elementwise_fma(xx, f2{wk.x, wk.y}, accp[o][0]);
                        if (NPR > 1) accp[o][1] = __builtin_elementwise_fma(xx, f2{wk.z, wk.w}, accp[o][1]);
                        if (NSG) accs[o][0] = fmaf(xv, MM == 1 ? wk.x : wk.z, accs[o][0]);
                    }
            }
        }
    };
    // one step of prefetch per quarter in registers: step k+1's loads are in flight under step k's
    // FMAs (LDS-DMA would not overlap: the compiler drains it before any LDS read)
    float4 r[CT_GT];
    const int nsteps = (Ct + CT_NQ * CT_CPQ - 1) / (CT_NQ * CT_CPQ);
    load(0, r);
    put(buf(0), r);
    __syncthreads();
    for (int k = 0; k < nsteps; ++k) {
        const bool more = k + 1 < nsteps;
        if (more) load(k + 1, r);
#pragma unroll
        for (int cl = 0; cl < CT_CPQ; ++cl) {
            compute(k, cl);
            __builtin_amdgcn_sched_barrier(0);   // one channel's neighbourhood live at a time
        }
        if (more) put(buf(k + 1), r);
        __syncthreads();
    }
    const int OH = 2 * a.IH, OW = 2 * a.IW;
    const int oy0 = 2 * (y0 + qy), ox0 = 2 * (x0 + qx);
    const bool xin = x0 + qx + 1 < a.IW;   // both input columns in range
    // argument fields read before the stores (after a store the compiler reloads them: ISA r04)
    float* const out = a.out;
    const float ap = a.act_param;
    // the activation as a template argument of the store loops (one switch outside them)
    auto with_act = [&](auto&& body) {
        switch (a.act) {
            case FFC_ACT_RELU: body([](float v) { return fmaxf(v, 0.0f); }); break;
            case FFC_ACT_LEAKY_RELU: body([ap](float v) { return v > 0.0f ? v : v * ap; }); break;
            case FFC_ACT_TANH: body([](float v) { return tanhf(v); }); break;
            case FFC_ACT_SIGMOID: body([](float v) { return 1.0f / (1.0f + expf(-v)); }); break;
            case FFC_ACT_GELU: body([](float v) { return 0.5f * v * (1.0f + erff(v * 0.70710678118654752f)); }); break;
            default: body([](float v) { return v; }); break;
        }
    };
    if (FFC_CT_ONECOMB && MM <= 3 && CT_NQ == 8 && CT_QT == 64 && a.comb == 1) {
        // 8 quarters of one wave each (the small-batch tiles): every quarter stores its partial sums
        // at once (the patch buffers are free after the last barrier), then wave w adds the output
        // rows (m, i) = w, w + 8, ... over the quarters in the serial combine's order
        // (((q0 + q1) + q2) + ...: the same rounding) and stores them -- one barrier instead of 14
        float* part = lds;   // [q][o * MM + m][QT]   (host: the dynamic LDS covers 8 * 16 * MM * 64 floats)
#pragma unroll
        for (int o = 0; o < 16; ++o)
#pragma unroll
            for (int m = 0; m < MM; ++m) part[((q * 16 + o) * MM + m) * CT_QT + tid] = get(o, m);
        __syncthreads();
        with_act([&](auto actf) {
            for (int u = q; u < 4 * MM; u += CT_NQ) {
                const int m = u >> 2, i = u & 3;
                const int oy = oy0 + i;
                const float bv = a.bias ? a.bias[m] : 0.0f;
                float v4[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int o = i * 4 + j;
                    float sacc = part[(o * MM + m) * CT_QT + tid];
#pragma unroll
                    for (int rq = 1; rq < CT_NQ; ++rq) sacc += part[((rq * 16 + o) * MM + m) * CT_QT + tid];
                    v4[j] = actf(sacc + bv);
                }
                if (oy >= OH) continue;
                float* row = out + (((size_t)b * M + m) * OH + oy) * OW + ox0;
                if (xin) {
                    *reinterpret_cast<float4*>(row) = make_float4(v4[0], v4[1], v4[2], v4[3]);
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (ox0 + j < OW) row[j] = v4[j];
                }
            }
        });
        return;
    }
    float* part = lds;
    if (FFC_CT_ONECOMB && MM <= 3 && CT_NQ != 8 && a.comb == 2) {
        // quarters 1 .. NQ-1 store their partial sums at once, quarter 0 adds them in quarter order
        // (the serial combine's rounding) after one barrier (host: LDS for (NQ - 1) * 16 * MM * QT floats)
        if (q != 0) {
#pragma unroll
            for (int o = 0; o < 16; ++o)
#pragma unroll
                for (int m = 0; m < MM; ++m) part[(((q - 1) * 16 + o) * MM + m) * CT_QT + tid] = get(o, m);
        }
        __syncthreads();
        if (q != 0) return;
        for (int rq = 1; rq < CT_NQ; ++rq) {
#pragma unroll
            for (int o = 0; o < 16; ++o)
#pragma unroll
                for (int m = 0; m < MM; ++m) add(o, m, part[(((rq - 1) * 16 + o) * MM + m) * CT_QT + tid]);
        }
    } else {
        // fixed-order combine of the quarters' partial sums: ((q0 + q1) + q2) + q3
        for (int rq = 1; rq < CT_NQ; ++rq) {
            if (q == rq) {
#pragma unroll
                for (int o = 0; o < 16; ++o)
#pragma unroll
                    for (int m = 0; m < MM; ++m) part[(o * MM + m) * CT_QT + tid] = get(o, m);
            }
            __syncthreads();
            if (q == 0) {
#pragma unroll
                for (int o = 0; o < 16; ++o)
#pragma unroll
                    for (int m = 0; m < MM; ++m) add(o, m, part[(o * MM + m) * CT_QT + tid]);
            }
            __syncthreads();
        }
        if (q != 0) return;
    }
    float bvs[MM];
#pragma unroll
    for (int m = 0; m < MM; ++m) bvs[m] = a.bias ? a.bias[m] : 0.0f;
    auto store = [&](auto actf) {
#pragma unroll
        for (int m = 0; m < MM; ++m) {
            const float bv = bvs[m];
            auto val = [&](int i, int j) { return actf(get(i * 4 + j, m) + bv); };
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int oy = oy0 + i;
                if (oy >= OH) continue;
                float* row = out + (((size_t)b * M + m) * OH + oy) * OW + ox0;
                if (xin) {
                    *reinterpret_cast<float4*>(row) = make_float4(val(i, 0), val(i, 1), val(i, 2), val(i, 3));
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (ox0 + j < OW) row[j] = val(i, j);
                }
            }
        }
    };
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
constexpr int T3 = 64;                      // output tile columns
constexpr int S3 = T3 + 8;                  // patch row: 18 float4 groups
constexpr int CMAX3 = 256;                  // channels (both segments)
// TR3 output rows per tile: 64 (one 512-thread workgroup per CU, 124 KB of LDS) or 32 (256 threads,
// ~64 KB with the weights sized to the channel count: two independent workgroups per CU, so one
// stages / waits on its barrier while the other computes).  Threads per half: (TR3 / 4) x 16.
template <int TR3>
struct Head3 {
    static constexpr int R3 = TR3 + 2;                        // patch rows (halo 1)
    static constexpr int G3 = R3 * (S3 / 4);                  // float4 groups per channel
    static constexpr int HT = (TR3 / 4) * 16;                 // threads per half
    static constexpr int GT3 = (G3 + HT - 1) / HT;            // groups per thread
    static constexpr int PB3 = G3 * 4;                        // floats per patch buffer
    static_assert(HT * 4 * 16 <= 4 * PB3, "combine area fits in the patch buffers");
};
size_t head3_lds_bytes(int tr) {
    const size_t pb = (size_t)(tr + 2) * (S3 / 4) * 4;
    return 4 * pb * sizeof(float);
}

// TF: each segment is read through its deferred transform a.tf[s] (ffc_in_tf): the producer's
// BN + activation + NoiseInjection applied as the patch goes to LDS, on in-image groups only (the
// zero padding belongs to the transformed tensor).  The head is VALU-bound, so GELU uses the
// branch-free gelu_as below instead of erff (whose two ranges diverge within a wave).
// three waves per SIMD (<= 168 VGPRs, a few spilled outside the FMA loop) instead of two at 182:
// fgan128 head 1.84 -> 1.77 ms (profiles/r04/aa)
#ifndef FFC_HEAD_WPE
#define FFC_HEAD_WPE 3
#endif
#define HEAD3_WPE __attribute__((amdgpu_waves_per_eu(FFC_HEAD_WPE)))
#ifndef FFC_HEAD_XCD
#define FFC_HEAD_XCD 1
#endif
template <int MM, bool TF, int TR3 = 64>
__global__ __launch_bounds__(2 * Head3<TR3>::HT) HEAD3_WPE void conv3x3_smallm_kernel(SmallMArgs a) {
    constexpr int R3 = Head3<TR3>::R3, G3 = Head3<TR3>::G3, HT = Head3<TR3>::HT, GT3 = Head3<TR3>::GT3;
    constexpr int PB3 = Head3<TR3>::PB3;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int half = __builtin_amdgcn_readfirstlane(threadIdx.x / HT), tid = threadIdx.x % HT;
    // XCD-aware order (FFC_HEAD_XCD): workgroups are dealt to the 8 XCDs round robin; remapped so
    // that each XCD runs consecutive tiles (a sample's tiles, whose halo rows overlap) through its L2:
    // fgan128 head HBM fetch 3.45 -> 2.20 GB per launch, 1.754 -> 1.716 ms (profiles/r04/ah)
    int bid = blockIdx.x;
#if FFC_HEAD_XCD
    if ((gridDim.x & 7) == 0) bid = (bid & 7) * (gridDim.x >> 3) + (bid >> 3);
#endif
    const int tx = bid % a.ntx;
    bid /= a.ntx;
    const int ty = bid % a.nty;
    const int b = bid / a.nty;
    const int y0 = ty * TR3, x0 = tx * T3;
    const int qy = 4 * (tid >> 4), qx = 4 * (tid & 15);   // this thread's 4x4 outputs (tile coords)
    const int M = a.M;
    const int nchunks = a.C[0] + (a.nseg > 1 ? a.C[1] : 0);   // one channel per chunk
    float* pbuf = lds;                                        // [2 buffers][2 halves][PB3]

    auto inimg = [&](int j) {
        const int n = j * HT + tid;
        const int g = n % (S3 / 4), pr = n / (S3 / 4);
        const int iy = y0 - 1 + pr, ix = x0 - 4 + 4 * g;
        return n < G3 && (unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW;
    };
    auto load = [&](int ci, float4 (&r)[GT3]) {
        const int s = ci < a.C[0] ? 0 : 1;
        const int c = s == 0 ? ci : ci - a.C[0];
        const float* x = a.x[s] + ((size_t)b * a.C[s] + c) * a.IH * a.IW;
#pragma unroll
        for (int j = 0; j < GT3; ++j) {
            const int n = j * HT + tid;
            const int g = n % (S3 / 4), pr = n / (S3 / 4);
            const int iy = y0 - 1 + pr, ix = x0 - 4 + 4 * g;
            r[j] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (inimg(j)) r[j] = *reinterpret_cast<const float4*>(x + (size_t)iy * a.IW + ix);
        }
    };
    // TF: this thread's noise float4s sit at the same patch positions for every channel of a segment,
    // so they are loaded once per segment (each half switches segment once)
    float4 nzr[TF ? GT3 : 1];
    int nz_seg = -1;
    auto put = [&](float* dst, float4 (&r)[GT3], int ci) {
        if constexpr (TF) {
            const int s = ci < a.C[0] ? 0 : 1;
            const int c = s == 0 ? ci : ci - a.C[0];
            const ffc_in_tf& t = a.tf[s];
            if (s != nz_seg) {
                const float* npl = t.noise ? t.noise + (size_t)b * a.IH * a.IW : nullptr;
#pragma unroll
                for (int j = 0; j < GT3; ++j) {
                    const int n = j * HT + tid;
                    const int g = n % (S3 / 4), pr = n / (S3 / 4);
                    const int iy = y0 - 1 + pr, ix = x0 - 4 + 4 * g;
                    nzr[j] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                    if (npl && inimg(j)) nzr[j] = *reinterpret_cast<const float4*>(npl + (size_t)iy * a.IW + ix);
                }
                nz_seg = s;
            }
            if (t.scale) {
                const float sc = t.scale[c], sh = t.shift[c];
                const float nw = t.noise ? t.noise_w[c] : 0.0f;
                const int act = t.act;
                const float p = t.act_param;
                auto tf4 = [&](auto actf) {
#pragma unroll
                    for (int j = 0; j < GT3; ++j) {
                        if (!inimg(j)) continue;
                        float4 v = r[j];
                        v = make_float4(actf(fmaf(v.x, sc, sh)), actf(fmaf(v.y, sc, sh)), actf(fmaf(v.z, sc, sh)),
                                        actf(fmaf(v.w, sc, sh)));
                        v.x = fmaf(nw, nzr[j].x, v.x);   // nzr is zero without noise
                        v.y = fmaf(nw, nzr[j].y, v.y);
                        v.z = fmaf(nw, nzr[j].z, v.z);
                        v.w = fmaf(nw, nzr[j].w, v.w);
                        r[j] = v;
                    }
                };
                if (act == FFC_ACT_GELU) {
#pragma unroll
                    for (int j = 0; j < GT3; ++j) {
                        if (!inimg(j)) continue;
                        const float4 v = r[j];
                        const f2 lo = gelu_as2(f2{fmaf(v.x, sc, sh), fmaf(v.y, sc, sh)});
                        const f2 hi = gelu_as2(f2{fmaf(v.z, sc, sh), fmaf(v.w, sc, sh)});
                        r[j] = make_float4(fmaf(nw, nzr[j].x, lo.x), fmaf(nw, nzr[j].y, lo.y),
                                           fmaf(nw, nzr[j].z, hi.x), fmaf(nw, nzr[j].w, hi.y));
                    }
                } else

                    tf4([act, p](float v) { return ffc::apply_act(v, act, p); });
            }
        }
#pragma unroll
        for (int j = 0; j < GT3; ++j) {
            const int n = j * HT + tid;
            if (n < G3) reinterpret_cast<float4*>(dst)[n] = r[j];
        }
    };
    auto buf = [&](int k) { return pbuf + ((k & 1) * 2 + half) * PB3; };

    // accumulators as column pairs (j, j+1): the FMAs run as v_pk_fma_f32 (two output columns against
    // one broadcast weight), half the VALU issue of scalar FMAs
    f2 acc2[MM][4][2];
#pragma unroll
    for (int m = 0; m < MM; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc2[m][i][j] = f2{0.0f, 0.0f};
#define ACC(m, i, j) (((j) & 1) ? acc2[m][i][(j) >> 1].y : acc2[m][i][(j) >> 1].x)

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
        // the channel's 9 M weights are wave-uniform: scalar loads straight from the (M, C_s, 3, 3)
        // tensor into SGPRs (no LDS broadcast reads: they cost the LDS return path 64 lanes x 16 B each)
        const int ws = ci < a.C[0] ? 0 : 1;
        const float* wsg = a.w[ws] + (ws == 0 ? ci : ci - a.C[0]) * 9;
        const int wms = a.C[ws] * 9;
#pragma unroll
        for (int m = 0; m < MM; ++m) {
            float k9[9];
#pragma unroll
            for (int t = 0; t < 9; ++t) k9[t] = wsg[m * wms + t];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int jp = 0; jp < 2; ++jp) {
                    f2 s2 = acc2[m][i][jp];
#pragma unroll
                    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                        for (int kx = 0; kx < 3; ++kx) {
                            const float w = k9[ky * 3 + kx];
                            s2 = __builtin_elementwise_fma(f2{v[i + ky][2 * jp + kx], v[i + ky][2 * jp + kx + 1]},
                                                           f2{w, w}, s2);
                        }
                    acc2[m][i][jp] = s2;
                }
        }
    };
    // one channel of prefetch in registers: channel k+1's loads are in flight under channel k's FMAs
    // (a second register set measured slower: 196 VGPRs, same occupancy)
    float4 r[GT3];
    if (half < nchunks) {
        load(half, r);
        put(buf(0), r, half);
    }
    __syncthreads();
    for (int k = 0; k < nsteps; ++k) {
        const int cn = 2 * (k + 1) + half;
        if (cn < nchunks) load(cn, r);
        compute(k);
        if (cn < nchunks) put(buf(k + 1), r, cn);
        __syncthreads();
    }
    // fixed-order combine of the two halves' partial sums (half 1 -> LDS -> half 0 adds)
    float* part = pbuf;   // HT threads x MM x 16 floats <= 4 * PB3
    if (half == 1) {
#pragma unroll
        for (int m = 0; m < MM; ++m)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) part[((m * 4 + i) * 4 + j) * HT + tid] = ACC(m, i, j);
    }
    __syncthreads();
    if (half == 1) return;
#pragma unroll
    for (int m = 0; m < MM; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int jp = 0; jp < 2; ++jp)
                acc2[m][i][jp] += f2{part[((m * 4 + i) * 4 + 2 * jp) * HT + tid],
                                     part[((m * 4 + i) * 4 + 2 * jp + 1) * HT + tid]};
    const int oy0 = y0 + qy, ox0 = x0 + qx;
    // argument fields read before the stores (after a store the compiler reloads them: ISA r04)
    float* const out = a.out;
    const int IH = a.IH, IW = a.IW;
    const bool xin = ox0 + 3 < IW;
    float bvs[MM];
#pragma unroll
    for (int m = 0; m < MM; ++m) bvs[m] = (a.bias && m < M) ? a.bias[m] : 0.0f;
    auto store = [&](auto actf) {
#pragma unroll
        for (int m = 0; m < MM; ++m) {
            if (m >= M) break;
            const float bv = bvs[m];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int oy = oy0 + i;
                if (oy >= IH) continue;
                float* row = out + (((size_t)b * M + m) * IH + oy) * IW + ox0;
                if (xin) {
                    *reinterpret_cast<float4*>(row) = make_float4(actf(ACC(m, i, 0) + bv), actf(ACC(m, i, 1) + bv),
                                                                  actf(ACC(m, i, 2) + bv), actf(ACC(m, i, 3) + bv));
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (ox0 + j < IW) row[j] = actf(ACC(m, i, j) + bv);
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
#undef ACC

}  // namespace

static __global__ void convt_smallm_pack_kernel(const float* __restrict__ w0, int C0, const float* __restrict__ w1,
                                         int C1, int M, float* __restrict__ wp) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (C0 + C1) * 64) return;
    const int ci = i >> 6, tap = (i >> 2) & 15, m = i & 3;
    const float* w = ci < C0 ? w0 : w1;
    const int c = ci < C0 ? ci : ci - C0;
    wp[i] = m < M ? w[((size_t)c * M + m) * 16 + tap] : 0.0f;
}

extern "C" size_t ffc_convt_smallm_pack_floats(int C0, int C1) {
    return C0 > 0 && C1 >= 0 ? ((size_t)C0 + (size_t)C1) * 64 : 0;
}

extern "C" int ffc_convt_smallm_pack(const float* w0, int C0, const float* w1, int C1, int M, float* wpack,
                                     void* stream) {
    FFC_CHECK_ARG(w0 && wpack && C0 > 0 && C1 >= 0 && (C1 == 0 || w1) && M >= 1 && M <= 4,
                  "ffc_convt_smallm_pack: bad args");
    const int n = (C0 + C1) * 64;
    hipLaunchKernelGGL(convt_smallm_pack_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, w0, C0,
                       w1, C1, M, wpack);
    return ffc::launch_status("ffc_convt_smallm_pack");
}

extern "C" int ffc_convt_k4s2_smallm(const float* x0, int C0, const float* x1, int C1, const float* wpack,
                                     const float* bias, int B, int IH, int IW, int M, float* out, int act,
                                     float act_param, void* stream) {
    FFC_CHECK_ARG(x0 && wpack && out && B > 0 && IH > 0 && IW > 0 && C0 > 0, "ffc_convt_k4s2_smallm: bad args");
    FFC_CHECK_ARG(M >= 1 && M <= 4, "ffc_convt_k4s2_smallm: 1 <= M <= 4");
    FFC_CHECK_ARG(!x1 || C1 > 0, "ffc_convt_k4s2_smallm: second segment");
    FFC_CHECK_ARG((reinterpret_cast<uintptr_t>(out) & 15) == 0 && (reinterpret_cast<uintptr_t>(wpack) & 15) == 0,
                  "ffc_convt_k4s2_smallm: output / packed weights not 16-B aligned");
    FFC_CHECK_ARG(C0 + (x1 ? C1 : 0) <= CT_CMAX, "ffc_convt_k4s2_smallm: at most 256 input channels");
    SmallMArgs a;
    a.x[0] = x0;
    a.w[0] = nullptr;
    a.C[0] = C0;
    a.x[1] = x1;
    a.w[1] = nullptr;
    a.C[1] = x1 ? C1 : 0;
    a.nseg = x1 ? 2 : 1;
    a.wpack = wpack;
    a.bias = bias;
    a.out = out;
    a.B = B;
    a.IH = IH;
    a.IW = IW;
    a.M = M;
    // fewer workgroups than CUs with 16-row tiles: 8-row tiles over 8 channel quarters
    const bool small = (long long)B * ((IH + CT_TR - 1) / CT_TR) * ((IW + CT_TT - 1) / CT_TT) < 256 && IH > 8;
    const int tr = small ? 8 : CT_TR, nq = small ? 8 : CT_NQ;
    a.nty = (IH + tr - 1) / tr;
    a.ntx = (IW + CT_TT - 1) / CT_TT;
    a.act = act;
    a.act_param = act_param;

    size_t lds = (size_t)2 * nq * CT_CPQ * (tr + 2) * CT_PS * sizeof(float);   // patch double buffer
    // quarter combine (convt_smallm_kernel): all 8 one-wave quarters at once when the grid is one
    // workgroup per CU or less (its LDS allows one per CU); else one barrier into quarter 0 while that
    // keeps two workgroups per CU (<= 80 KB); else the serial combine
    const size_t qt = (size_t)(CT_TT / 2) * (tr / 2);
    const size_t comb_all = (size_t)nq * 16 * M * qt * sizeof(float);
    const size_t comb_q0 = (size_t)(nq - 1) * 16 * M * qt * sizeof(float);
    a.comb = 0;   // M = 4: the serial combine (the one-barrier forms spill registers there)
    if (M > 3) {
    } else if (nq == 8 && qt == 64 && (long long)B * a.nty * a.ntx <= 256 && comb_all <= 160 * 1024) {
        a.comb = 1;
        lds = std::max(lds, comb_all);
    } else if (nq != 8 && comb_q0 <= 80 * 1024) {
        a.comb = 2;
        lds = std::max(lds, comb_q0);
    }
    const unsigned grid = (unsigned)B * a.nty * a.ntx;
    // M is a template parameter: no runtime m < M branches in the FMA body
    typedef void (*CtKernel)(SmallMArgs);
    static const CtKernel kernels[2][2][4] = {
        {{convt_smallm_kernel<1, false>, convt_smallm_kernel<2, false>, convt_smallm_kernel<3, false>,
          convt_smallm_kernel<4, false>},
         {convt_smallm_kernel<1, true>, convt_smallm_kernel<2, true>, convt_smallm_kernel<3, true>,
          convt_smallm_kernel<4, true>}},
        {{convt_smallm_kernel<1, false, 8, 8>, convt_smallm_kernel<2, false, 8, 8>, convt_smallm_kernel<3, false, 8, 8>,
          convt_smallm_kernel<4, false, 8, 8>},
         {convt_smallm_kernel<1, true, 8, 8>, convt_smallm_kernel<2, true, 8, 8>, convt_smallm_kernel<3, true, 8, 8>,
          convt_smallm_kernel<4, true, 8, 8>}}};
    const int vec = IW % 4 == 0 ? 1 : 0;
    auto k = kernels[small][vec][M - 1];
    static bool raised[2][2][5] = {};
    if (!raised[small][vec][M]) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024) != hipSuccess) {
            ffc::set_error("ffc_convt_k4s2_smallm: hipFuncSetAttribute failed");
            return FFC_E_LAUNCH;
        }
        raised[small][vec][M] = true;
    }
    hipLaunchKernelGGL(k, dim3(grid), dim3((CT_TT / 2) * (tr / 2) * nq), lds, (hipStream_t)stream, a);
    return ffc::launch_status("ffc_convt_k4s2_smallm");
}

static int conv3x3_smallm_launch(const float* x0, int C0, const float* w0, const float* x1, int C1,
                                 const float* w1, const float* bias, int B, int H, int W, int M, float* out,
                                 int act, float act_param, const ffc_in_tf* tf0, const ffc_in_tf* tf1,
                                 void* stream) {
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
    a.wpack = nullptr;
    a.bias = bias;
    a.out = out;
    a.B = B;
    a.IH = H;
    a.IW = W;
    a.M = M;
    // tile rows: 32 (two workgroups per CU; measured: fgan128 B = 512 head 2.25 -> 2.11 ms, B = 64 neutral,
    // profiles/r02/s15); FFC_HEAD_TR=64 restores the full-height tile for A/B runs
    static const int tr = [] {
        const char* e = std::getenv("FFC_HEAD_TR");
        return e && std::atoi(e) == 64 ? 64 : 32;
    }();
    a.nty = (H + tr - 1) / tr;
    a.ntx = (W + T3 - 1) / T3;
    a.act = act;
    a.act_param = act_param;
    FFC_CHECK_ARG(C0 + (x1 ? C1 : 0) <= CMAX3, "ffc_conv3x3_smallm: at most 256 input channels");
    const ffc_in_tf none = {nullptr, nullptr, 0, 0.0f, nullptr, nullptr};
    const ffc_in_tf* tfs[2] = {tf0, x1 ? tf1 : nullptr};
    const bool tf = tfs[0] || tfs[1];
    for (int s = 0; s < 2; ++s) {
        const ffc_in_tf* t = tfs[s];
        FFC_CHECK_ARG(!t || (t->scale && t->shift && (!t->noise || t->noise_w)),
                      "ffc_conv3x3_smallm_tf: a transform needs scale, shift (and noise_w with noise)");
        FFC_CHECK_ARG(!t || !t->noise || (reinterpret_cast<uintptr_t>(t->noise) & 15) == 0,
                      "ffc_conv3x3_smallm_tf: noise not 16-B aligned");
        a.tf[s] = t ? *t : none;
    }
    const int nchunks = C0 + (x1 ? C1 : 0);
    const size_t lds = head3_lds_bytes(tr);
    const unsigned grid = (unsigned)B * a.nty * a.ntx;
    // M is a template parameter: no runtime m < M branches in the FMA body
    typedef void (*C3Kernel)(SmallMArgs);
    static const C3Kernel kernels[2][2][4] = {
        {{conv3x3_smallm_kernel<1, false>, conv3x3_smallm_kernel<2, false>, conv3x3_smallm_kernel<3, false>,
          conv3x3_smallm_kernel<4, false>},
         {conv3x3_smallm_kernel<1, true>, conv3x3_smallm_kernel<2, true>, conv3x3_smallm_kernel<3, true>,
          conv3x3_smallm_kernel<4, true>}},
        {{conv3x3_smallm_kernel<1, false, 32>, conv3x3_smallm_kernel<2, false, 32>,
          conv3x3_smallm_kernel<3, false, 32>, conv3x3_smallm_kernel<4, false, 32>},
         {conv3x3_smallm_kernel<1, true, 32>, conv3x3_smallm_kernel<2, true, 32>, conv3x3_smallm_kernel<3, true, 32>,
          conv3x3_smallm_kernel<4, true, 32>}}};
    const int ti = tr == 32 ? 1 : 0;
    auto k = kernels[ti][tf ? 1 : 0][M - 1];
    static bool raised[2][2][5] = {};
    if (!raised[ti][tf][M]) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024) != hipSuccess) {
            ffc::set_error("ffc_conv3x3_smallm: hipFuncSetAttribute failed");
            return FFC_E_LAUNCH;
        }
        raised[ti][tf][M] = true;
    }
    hipLaunchKernelGGL(k, dim3(grid), dim3(tr == 32 ? 2 * Head3<32>::HT : 2 * Head3<64>::HT), lds,
                       (hipStream_t)stream, a);
    return ffc::launch_status("ffc_conv3x3_smallm");
}

extern "C" int ffc_conv3x3_smallm(const float* x0, int C0, const float* w0, const float* x1, int C1,
                                  const float* w1, const float* bias, int B, int H, int W, int M, float* out,
                                  int act, float act_param, void* stream) {
    return conv3x3_smallm_launch(x0, C0, w0, x1, C1, w1, bias, B, H, W, M, out, act, act_param, nullptr, nullptr,
                                 stream);
}

extern "C" int ffc_conv3x3_smallm_tf(const float* x0, int C0, const float* w0, const float* x1, int C1,
                                     const float* w1, const float* bias, int B, int H, int W, int M, float* out,
                                     int act, float act_param, const ffc_in_tf* tf0, const ffc_in_tf* tf1,
                                     void* stream) {
    return conv3x3_smallm_launch(x0, C0, w0, x1, C1, w1, bias, B, H, W, M, out, act, act_param, tf0, tf1, stream);
}
