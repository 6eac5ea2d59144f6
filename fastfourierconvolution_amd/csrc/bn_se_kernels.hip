// Batch-norm statistics / apply and the SE gate for gfx950.
//
// BN: partial slabs {n, mean, M2} (written by the GEMM and FU epilogues) are merged in
// fp64 in a fixed order -> deterministic; nn.BatchNorm2d running-stat semantics
// (torch/nn/modules/batchnorm.py as called from layers/ffc/*.py) are reproduced exactly.
// SE: SELayer (layers/ffc/spectral_transform.py:12-28).
#include "ffc_internal.h"
#include "bn_common.h"

#include <algorithm>
#include <cstdlib>

#include <cmath>

namespace {

constexpr int RED_THREADS = 256;

// whole-wave fp64 sum, bit-identical in every lane: the DPP / v_permlane*_swap tree of bn_common.h
// (ffc::group_sum_f64<64>) -- the reductions stay in the VALU; the ds_bpermute tree it replaces
// (__shfl_xor, two LDS-pipe round trips per level and double) was most of a finalize launch's
// latency chain.  FFC_BN_SHFL=1 keeps the __shfl_xor tree (A/B).
#ifndef FFC_BN_SHFL
#define FFC_BN_SHFL 0
#endif
__device__ __forceinline__ double wave_sum_f64(double v) {
    if constexpr (FFC_BN_SHFL) {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
        return v;
    }
    return ffc::group_sum_f64<64>(v);
}

// one block per channel: merge rows of a {n, mean, M2} slab into fp64 raw moments {n, sum, sumsq}
// (fixed order: strided per-thread sums, a shuffle tree per wave, the waves in order), returned
// in thread 0's m[] and stored to out3.  Latency-bound (a few hundred rows): every thread keeps
// its loads in flight (unrolled by 4) and the tree needs one barrier.
__device__ void reduce_channel(const float4* __restrict__ slab, int nrows, int C, int c, double* out3, double (&m)[3]) {
    __shared__ double sh[RED_THREADS / 64][3];
    double n = 0.0, s = 0.0, q = 0.0;
    int r = threadIdx.x;
    for (; r + 3 * RED_THREADS < nrows; r += 4 * RED_THREADS) {
        float4 e[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) e[u] = slab[(size_t)(r + u * RED_THREADS) * C + c];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const double en = e[u].x, em = e[u].y;
            n += en;
            s += en * em;
            q += (double)e[u].z + en * em * em;
        }
    }
    for (; r < nrows; r += RED_THREADS) {
        const float4 e = slab[(size_t)r * C + c];
        const double en = e.x, em = e.y;
        n += en;
        s += en * em;
        q += (double)e.z + en * em * em;
    }
    n = wave_sum_f64(n);
    s = wave_sum_f64(s);
    q = wave_sum_f64(q);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sh[w][0] = n;
        sh[w][1] = s;
        sh[w][2] = q;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        m[0] = m[1] = m[2] = 0.0;
#pragma unroll
        for (int i = 0; i < RED_THREADS / 64; ++i) {
            m[0] += sh[i][0];
            m[1] += sh[i][1];
            m[2] += sh[i][2];
        }
        out3[0] = m[0];
        out3[1] = m[1];
        out3[2] = m[2];
    }
}

struct FinalizeArgs {
    const float* gamma;
    const float* beta;
    float* running_mean;
    float* running_var;
    int64_t* nbt;
    int use_batch_stats, update_running;
    int bump_here;   // momentum given: nobody reads num_batches_tracked, so one thread bumps it in-kernel
    float momentum, eps, count_mult;
    float* scale;
    float* shift;
};

// the per-channel BN parameters finalize_channel reads, loaded up front (their latency then
// overlaps the slab reduction)
struct FinalizeIn {
    float g, bb, rm, rv;
    int64_t nbt;
};

__device__ __forceinline__ FinalizeIn finalize_load(int c, const FinalizeArgs& a) {
    FinalizeIn in;
    in.g = a.gamma ? a.gamma[c] : 1.0f;
    in.bb = a.beta ? a.beta[c] : 0.0f;
    const bool need_running = !a.use_batch_stats || a.update_running;
    in.rm = need_running ? a.running_mean[c] : 0.0f;
    in.rv = need_running ? a.running_var[c] : 0.0f;
    in.nbt = a.update_running && a.momentum < 0.0f ? *a.nbt : 0;
    return in;
}

__device__ void finalize_channel(const double* m3, int c, const FinalizeArgs& a, const FinalizeIn& in) {
    float mean, var;
    if (a.use_batch_stats) {
        const double n = m3[0];
        const double mu = m3[1] / n;
        double v = m3[2] / n - mu * mu;
        if (v < 0.0) v = 0.0;
        mean = (float)mu;
        var = (float)v;
        if (a.update_running) {
            float f = a.momentum;
            if (f < 0.0f) f = 1.0f / (float)(in.nbt + 1);  // momentum=None: cumulative average
            const double nfull = n * (double)a.count_mult;
            const double unb = nfull > 1.0 ? v * nfull / (nfull - 1.0) : v;
            // explicit fmaf: the single, batched and in-kernel-fold finalizes then round identically
            // whatever contraction the compiler picks per kernel (a -fno-slp-vectorize build broke
            // their bit-identity, profiles/r03/s2l/tests_noslp.log)
            a.running_mean[c] = fmaf(f, mean, (1.0f - f) * in.rm);
            a.running_var[c] = fmaf(f, (float)unb, (1.0f - f) * in.rv);
        }
    } else {
        mean = in.rm;
        var = in.rv;
    }
    const float inv = 1.0f / sqrtf(var + a.eps);
    const float sc = in.g * inv;
    a.scale[c] = sc;
    a.shift[c] = fmaf(-mean, sc, in.bb);
}

__device__ void finalize_channel(const double* m3, int c, const FinalizeArgs& a) {
    finalize_channel(m3, c, a, finalize_load(c, a));
}

__global__ void bn_reduce_kernel(const float4* __restrict__ slab, int nrows, int C, double* moments) {
    double m[3];
    reduce_channel(slab, nrows, C, blockIdx.x, moments + 3 * blockIdx.x, m);
}

__global__ void bn_finalize_kernel(const double* __restrict__ moments, int C, FinalizeArgs a) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c < C) finalize_channel(moments + 3 * c, c, a);
    if (a.bump_here && c == 0) *a.nbt += 1;
}

// nbt is bumped after every block has read it (stream order: separate tiny kernel)
__global__ void bn_bump_kernel(int64_t* nbt) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *nbt += 1;
}

__global__ void bn_reduce_finalize_kernel(const float4* __restrict__ slab, int nrows, int C, double* moments,
                                          FinalizeArgs a) {
    const int c = blockIdx.x;
    FinalizeIn in = {};
    if (threadIdx.x == 0) in = finalize_load(c, a);
    double m[3];
    reduce_channel(slab, nrows, C, c, moments + 3 * c, m);
    if (threadIdx.x == 0) finalize_channel(m, c, a, in);
    if (a.bump_here && c == 0 && threadIdx.x == 0) *a.nbt += 1;
}

__global__ void bn_act_kernel(const float* __restrict__ x, float* __restrict__ y, int C, int HW, long long total4,
                              const float* __restrict__ scale, const float* __restrict__ shift, int act, float p) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += stride) {
        const long long e = i * 4;
        float4 v = reinterpret_cast<const float4*>(x)[i];
        float r[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = (int)(((e + j) / HW) % C);
            r[j] = ffc::apply_act(fmaf(r[j], scale[c], shift[c]), act, p);
        }
        reinterpret_cast<float4*>(y)[i] = make_float4(r[0], r[1], r[2], r[3]);
    }
}

__global__ void bn_act_scalar_kernel(const float* __restrict__ x, float* __restrict__ y, int C, int HW,
                                     long long total, const float* __restrict__ scale,
                                     const float* __restrict__ shift, int act, float p) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const int c = (int)((i / HW) % C);
        y[i] = ffc::apply_act(fmaf(x[i], scale[c], shift[c]), act, p);
    }
}

// SE gate: one block per sample; 256 threads
__global__ void se_gate_kernel(const float* __restrict__ x, int C, int H, int W, int pool,
                               const float* __restrict__ w1, const float* __restrict__ w2, int hid,
                               float* __restrict__ gate) {
    extern __shared__ float sm[];
    float* mean = sm;       // C
    float* hv = sm + C;     // hid
    const int b = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int Hc = pool ? (H / 2) * 2 : H;  // AvgPool2d(2,2) floors: odd last row/col dropped
    const int Wc = pool ? (W / 2) * 2 : W;
    const float inv = 1.0f / (float)(Hc * Wc);
    for (int c = wave; c < C; c += nw) {
        const float* p = x + ((size_t)b * C + c) * H * W;
        float s = 0.0f;
        for (int i = lane; i < Hc * Wc; i += 64) {
            const int yy = i / Wc, xx = i - yy * Wc;
            s += p[yy * W + xx];
        }
        s = ffc::wave_sum(s);
        if (lane == 0) mean[c] = s * inv;
    }
    __syncthreads();
    for (int j = threadIdx.x; j < hid; j += blockDim.x) {
        float s = 0.0f;
        for (int c = 0; c < C; ++c) s = fmaf(w1[(size_t)j * C + c], mean[c], s);
        hv[j] = fmaxf(s, 0.0f);
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        float s = 0.0f;
        for (int j = 0; j < hid; ++j) s = fmaf(w2[(size_t)c * hid + j], hv[j], s);
        gate[(size_t)b * C + c] = 1.0f / (1.0f + expf(-s));
    }
}

// BN scale/shift + activation (+ NoiseInjection) over whole planes: every block covers one chunk
// of one (b, c) plane, so the channel is computed once per block (no per-element division).
// out = act(x*scale[c] + shift[c]) [+ noise_w[c] * noise[b, hw]]   (layers/noise_injection.py:25-32)
constexpr int PLANE_CHUNK4 = 1024;   // float4 per block: 256 threads x 4
__global__ __launch_bounds__(256) void bn_act_plane_kernel(const float4* __restrict__ x, float4* __restrict__ y,
                                                           int C, int HW4, int chunks,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift, int act, float p,
                                                           const float* __restrict__ noise_w,
                                                           const float4* __restrict__ noise) {
    const int plane = blockIdx.x / chunks;
    const int chunk = blockIdx.x - plane * chunks;
    const int c = plane % C, b = plane / C;
    const float sc = scale[c], sh = shift[c];
    const float nw = noise_w ? noise_w[c] : 0.0f;
    const size_t base = (size_t)plane * HW4;
    const float4* nz = noise ? noise + (size_t)b * HW4 : nullptr;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = chunk * PLANE_CHUNK4 + u * 256 + threadIdx.x;
        if (i < HW4) {
            const float4 v = x[base + i];
            float4 r = make_float4(ffc::apply_act(fmaf(v.x, sc, sh), act, p), ffc::apply_act(fmaf(v.y, sc, sh), act, p),
                                   ffc::apply_act(fmaf(v.z, sc, sh), act, p), ffc::apply_act(fmaf(v.w, sc, sh), act, p));
            if (nz) {
                const float4 n = nz[i];
                r.x = fmaf(nw, n.x, r.x);
                r.y = fmaf(nw, n.y, r.y);
                r.z = fmaf(nw, n.z, r.z);
                r.w = fmaf(nw, n.w, r.w);
            }
            y[base + i] = r;
        }
    }
}

// SE gate for large planes, stage 1: one wave per (b, c) plane, float4 loads -> plane mean
// (the per-sample kernel above leaves most CUs idle when B is small and the planes large)
__global__ void se_mean_kernel(const float4* __restrict__ x, int planes, int HW4, float inv, float* __restrict__ mean) {
    const int lane = threadIdx.x & 63;
    const int p = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (p >= planes) return;
    const float4* src = x + (size_t)p * HW4;
    float s0 = 0.0f, s1 = 0.0f;
    int i = lane;
    for (; i + 64 < HW4; i += 128) {
        const float4 a = src[i], b = src[i + 64];
        s0 += (a.x + a.y) + (a.z + a.w);
        s1 += (b.x + b.y) + (b.z + b.w);
    }
    if (i < HW4) {
        const float4 a = src[i];
        s0 += (a.x + a.y) + (a.z + a.w);
    }
    const float s = ffc::wave_sum(s0 + s1);
    if (lane == 0) mean[p] = s * inv;
}

// stage 2: per sample, gate = sigmoid(W2 relu(W1 mean))
__global__ void se_fc_kernel(const float* means, int C, const float* __restrict__ w1,
                             const float* __restrict__ w2, int hid, float* gate) {
    extern __shared__ float sm[];
    float* mean = sm;
    float* hv = sm + C;
    const int b = blockIdx.x;
    for (int c = threadIdx.x; c < C; c += blockDim.x) mean[c] = means[(size_t)b * C + c];
    __syncthreads();
    for (int j = threadIdx.x; j < hid; j += blockDim.x) {
        float s = 0.0f;
        for (int c = 0; c < C; ++c) s = fmaf(w1[(size_t)j * C + c], mean[c], s);
        hv[j] = fmaxf(s, 0.0f);
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        float s = 0.0f;
        for (int j = 0; j < hid; ++j) s = fmaf(w2[(size_t)c * hid + j], hv[j], s);
        gate[(size_t)b * C + c] = 1.0f / (1.0f + expf(-s));
    }
}

// ---- two-level reduction of large slabs (thousands of rows: the fgan128 layers at B = 512).  The
// one-block-per-channel kernel above reads one float4 per lane from a different row (a 16-byte
// piece of 64 cache lines per load) and runs C blocks; here a block takes 16 channels x a row range
// (lane = 16 rg + oc: every load is 4 rows x 256 contiguous bytes) and ~512 blocks cover the slab,
// writing fp64 partials {n, sum, sumsq} to the scratch behind `moments`; the second kernel merges the
// S partials of a channel in a fixed order (lane-strided sums, one shuffle tree) and finalizes.
constexpr int RED2_MIN_ROWS = 1024;   // FFC_BN_RED2_MIN overrides (A/B runs)
int red2_min_rows() {
    static const int v = [] {
        const char* e = std::getenv("FFC_BN_RED2_MIN");
        return e && *e ? std::max(1, std::atoi(e)) : RED2_MIN_ROWS;
    }();
    return v;
}

__global__ __launch_bounds__(256) void bn_partial16_kernel(const float4* __restrict__ slab, int nrows, int C, int S,
                                                           double* __restrict__ ws) {
    const int cg = blockIdx.x, sp = blockIdx.y;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int oc = lane & 15, rgb = wave * 4 + (lane >> 4);   // 16 row groups per block
    const int c = cg * 16 + oc;
    const int cc = c < C ? c : C - 1;
    const int r_lo = (int)((long long)sp * nrows / S), r_hi = (int)((long long)(sp + 1) * nrows / S);
    double n = 0.0, s = 0.0, q = 0.0;
    int r = r_lo + rgb;
    for (; r + 48 < r_hi; r += 64) {   // four rows in flight per lane
        float4 e[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) e[u] = slab[(size_t)(r + 16 * u) * C + cc];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const double en = e[u].x, em = e[u].y;
            n += en;
            s += en * em;
            q += (double)e[u].z + en * em * em;
        }
    }
    for (; r < r_hi; r += 16) {
        const float4 e = slab[(size_t)r * C + cc];
        const double en = e.x, em = e.y;
        n += en;
        s += en * em;
        q += (double)e.z + en * em * em;
    }
    // the 4 row groups of the wave: v + v(lane ^ 16), then ^ 32, on v_permlane16/32_swap (the same sums
    // as the __shfl_xor pairs, without the ds_bpermute round trips)
    n = ffc::permlane_sum_f64<true>(n);
    s = ffc::permlane_sum_f64<true>(s);
    q = ffc::permlane_sum_f64<true>(q);
    n = ffc::permlane_sum_f64<false>(n);
    s = ffc::permlane_sum_f64<false>(s);
    q = ffc::permlane_sum_f64<false>(q);
    __shared__ double sh[4][16][3];
    if (lane < 16) {
        sh[wave][oc][0] = n;
        sh[wave][oc][1] = s;
        sh[wave][oc][2] = q;
    }
    __syncthreads();
    if (threadIdx.x < 16 && c < C) {
        double m3[3] = {0.0, 0.0, 0.0};
#pragma unroll
        for (int w = 0; w < 4; ++w)
#pragma unroll
            for (int i = 0; i < 3; ++i) m3[i] += sh[w][threadIdx.x][i];
        double* d = ws + ((size_t)sp * C + c) * 3;
        d[0] = m3[0];
        d[1] = m3[1];
        d[2] = m3[2];
    }
}

// one wave per channel: the S partials in a fixed order -> moments (+ finalize)
__global__ __launch_bounds__(64) void bn_merge_kernel(const double* __restrict__ ws, int S, int C, double* moments,
                                                      int finalize, FinalizeArgs a) {
    const int c = blockIdx.x, lane = threadIdx.x;
    FinalizeIn in = {};
    if (finalize && lane == 0) in = finalize_load(c, a);
    double n = 0.0, s = 0.0, q = 0.0;
    for (int sp = lane; sp < S; sp += 64) {
        const double* d = ws + ((size_t)sp * C + c) * 3;
        n += d[0];
        s += d[1];
        q += d[2];
    }
    n = wave_sum_f64(n);
    s = wave_sum_f64(s);
    q = wave_sum_f64(q);
    if (lane == 0) {
        double* m = moments + 3 * c;
        m[0] = n;
        m[1] = s;
        m[2] = q;
        if (finalize) {
            const double m3[3] = {n, s, q};
            finalize_channel(m3, c, a, in);
            if (a.bump_here && c == 0) *a.nbt += 1;
        }
    }
}

int red2_splits(int nrows, int C) {
    if (nrows < red2_min_rows()) return 0;
    const int ncg = (C + 15) / 16;
    return std::max(1, std::min(nrows / 64, (512 + ncg - 1) / ncg));
}

// ---- batched forms: one launch for the BNs of a layer (items located by block-index prefix sums)
struct RfBatch {
    const float4* slab[FFC_MAX_BN_BATCH];
    double* moments[FFC_MAX_BN_BATCH];
    FinalizeArgs fa[FFC_MAX_BN_BATCH];
    int nrows[FFC_MAX_BN_BATCH], C[FFC_MAX_BN_BATCH];
    int off[FFC_MAX_BN_BATCH + 1];
    int n;
};

__global__ void bn_reduce_finalize_batch_kernel(RfBatch a) {
    int it = 0;
    while (it + 1 < a.n && (int)blockIdx.x >= a.off[it + 1]) ++it;
    const int c = blockIdx.x - a.off[it];
    FinalizeIn in = {};
    if (threadIdx.x == 0) in = finalize_load(c, a.fa[it]);
    double m[3];
    reduce_channel(a.slab[it], a.nrows[it], a.C[it], c, a.moments[it] + 3 * c, m);
    if (threadIdx.x == 0) finalize_channel(m, c, a.fa[it], in);
    if (a.fa[it].bump_here && c == 0 && threadIdx.x == 0) *a.fa[it].nbt += 1;
}

struct ApplyBatch {
    const float4* x[FFC_MAX_BN_BATCH];
    float4* y[FFC_MAX_BN_BATCH];
    const float* scale[FFC_MAX_BN_BATCH];
    const float* shift[FFC_MAX_BN_BATCH];
    const float* noise_w[FFC_MAX_BN_BATCH];
    const float4* noise[FFC_MAX_BN_BATCH];
    float* psum[FFC_MAX_BN_BATCH];
    int C[FFC_MAX_BN_BATCH], HW4[FFC_MAX_BN_BATCH], chunks[FFC_MAX_BN_BATCH], act[FFC_MAX_BN_BATCH];
    float p[FFC_MAX_BN_BATCH];
    int off[FFC_MAX_BN_BATCH + 1];
    int n;
};

// bn_act_plane_kernel over several tensors: block -> (item, plane, chunk)
__global__ __launch_bounds__(256) void bn_act_plane_batch_kernel(ApplyBatch a) {
    int it = 0;
    while (it + 1 < a.n && (int)blockIdx.x >= a.off[it + 1]) ++it;
    const int bid = blockIdx.x - a.off[it];
    const int chunks = a.chunks[it], HW4 = a.HW4[it];
    const int plane = bid / chunks, chunk = bid - plane * chunks;
    const int c = plane % a.C[it], b = plane / a.C[it];
    const float sc = a.scale[it][c], sh = a.shift[it][c];
    const float nw = a.noise_w[it] ? a.noise_w[it][c] : 0.0f;
    const int act = a.act[it];
    const float p = a.p[it];
    const size_t base = (size_t)plane * HW4;
    const float4* nz = a.noise[it] ? a.noise[it] + (size_t)b * HW4 : nullptr;
    const float4* x = a.x[it];
    float4* y = a.y[it];
    float* const psum = a.psum[it];
    float ts = 0.0f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = chunk * PLANE_CHUNK4 + u * 256 + threadIdx.x;
        if (i < HW4) {
            const float4 v = x[base + i];
            float4 r = make_float4(ffc::apply_act(fmaf(v.x, sc, sh), act, p), ffc::apply_act(fmaf(v.y, sc, sh), act, p),
                                   ffc::apply_act(fmaf(v.z, sc, sh), act, p), ffc::apply_act(fmaf(v.w, sc, sh), act, p));
            if (nz) {
                const float4 n = nz[i];
                r.x = fmaf(nw, n.x, r.x);
                r.y = fmaf(nw, n.y, r.y);
                r.z = fmaf(nw, n.z, r.z);
                r.w = fmaf(nw, n.w, r.w);
            }
            y[base + i] = r;
            ts += (r.x + r.y) + (r.z + r.w);
        }
    }
    if (psum) {   // the chunk's sum of y: waves' halves (DPP), then the 8 half sums in a fixed order
        __shared__ float hsum[8];
        const float hs = ffc::half_wave_sum(ts);
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        if (lane == 0 || lane == 32) hsum[2 * wave + (lane >> 5)] = hs;
        __syncthreads();
        if (threadIdx.x == 0) {
            float s = 0.0f;
#pragma unroll
            for (int k = 0; k < 8; ++k) s += hsum[k];
            psum[(size_t)plane * chunks + chunk] = s;
        }
    }
}

// SE gate from the plane-chunk sums of ffc_bn_act_apply_batch: one block per sample
__global__ void se_fc_sums_kernel(const float* __restrict__ sums, int chunks, int C, float inv,
                                  const float* __restrict__ w1, const float* __restrict__ w2, int hid,
                                  float* __restrict__ gate) {
    extern __shared__ float sm[];
    float* mean = sm;
    float* hv = sm + C;
    const int b = blockIdx.x;
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        const float* q = sums + ((size_t)b * C + c) * chunks;
        float s = 0.0f;
        for (int k = 0; k < chunks; ++k) s += q[k];
        mean[c] = s * inv;
    }
    __syncthreads();
    for (int j = threadIdx.x; j < hid; j += blockDim.x) {
        float s = 0.0f;
        for (int c = 0; c < C; ++c) s = fmaf(w1[(size_t)j * C + c], mean[c], s);
        hv[j] = fmaxf(s, 0.0f);
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        float s = 0.0f;
        for (int j = 0; j < hid; ++j) s = fmaf(w2[(size_t)c * hid + j], hv[j], s);
        gate[(size_t)b * C + c] = 1.0f / (1.0f + expf(-s));
    }
}

}  // namespace

extern "C" size_t ffc_bn_reduce_ws_doubles(int nrows, int C) {
    if (nrows <= 0 || C <= 0) return 0;
    return (size_t)red2_splits(nrows, C) * (size_t)C * 3;
}

// large slabs: partials into the scratch behind moments, then the merge (finalize when fa != null)
static void bn_reduce2(const float* slab, int nrows, int C, double* moments, const FinalizeArgs* fa,
                       hipStream_t stream) {
    const int S = red2_splits(nrows, C);
    double* ws = moments + 3 * (size_t)C;
    hipLaunchKernelGGL(bn_partial16_kernel, dim3((C + 15) / 16, S), dim3(256), 0, stream,
                       reinterpret_cast<const float4*>(slab), nrows, C, S, ws);
    FinalizeArgs a = fa ? *fa : FinalizeArgs{};
    hipLaunchKernelGGL(bn_merge_kernel, dim3(C), dim3(64), 0, stream, ws, S, C, moments, fa ? 1 : 0, a);
}

extern "C" int ffc_bn_reduce(const float* slab, int nrows, int C, double* moments, void* stream) {
    FFC_CHECK_ARG(slab && moments && nrows > 0 && C > 0, "ffc_bn_reduce: bad args");
    if (red2_splits(nrows, C)) {
        bn_reduce2(slab, nrows, C, moments, nullptr, (hipStream_t)stream);
        return ffc::launch_status("ffc_bn_reduce");
    }
    hipLaunchKernelGGL(bn_reduce_kernel, dim3(C), dim3(RED_THREADS), 0, (hipStream_t)stream,
                       reinterpret_cast<const float4*>(slab), nrows, C, moments);
    return ffc::launch_status("ffc_bn_reduce");
}

static FinalizeArgs make_finalize(const float* gamma, const float* beta, float* rm, float* rv, int64_t* nbt,
                                  int use_batch_stats, int update_running, float momentum, float eps,
                                  float count_mult, float* scale, float* shift) {
    FinalizeArgs a;
    a.gamma = gamma;
    a.beta = beta;
    a.running_mean = rm;
    a.running_var = rv;
    a.nbt = nbt;
    a.use_batch_stats = use_batch_stats;
    a.update_running = update_running;
    a.bump_here = update_running && use_batch_stats && momentum >= 0.0f;
    a.momentum = momentum;
    a.eps = eps;
    a.count_mult = count_mult;
    a.scale = scale;
    a.shift = shift;
    return a;
}

extern "C" int ffc_bn_finalize(const double* moments, int C, const float* gamma, const float* beta,
                               float* running_mean, float* running_var, int64_t* num_batches_tracked,
                               int use_batch_stats, int update_running, float momentum, float eps, float count_mult,
                               float* scale, float* shift, void* stream) {
    FFC_CHECK_ARG(C > 0 && scale && shift, "ffc_bn_finalize: bad args");
    FFC_CHECK_ARG(!use_batch_stats || moments, "ffc_bn_finalize: batch stats need moments");
    FFC_CHECK_ARG(use_batch_stats || (running_mean && running_var), "ffc_bn_finalize: eval needs running stats");
    FFC_CHECK_ARG(!update_running || (running_mean && running_var && num_batches_tracked),
                  "ffc_bn_finalize: update needs running buffers");
    FinalizeArgs a = make_finalize(gamma, beta, running_mean, running_var, num_batches_tracked, use_batch_stats,
                                   update_running, momentum, eps, count_mult, scale, shift);
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, moments, C, a);
    // momentum=None (cumulative average) reads num_batches_tracked in every block: bump after them
    if (update_running && use_batch_stats && !a.bump_here)
        hipLaunchKernelGGL(bn_bump_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, num_batches_tracked);
    return ffc::launch_status("ffc_bn_finalize");
}

// fused single-rank path (no cross-rank all-reduce between reduce and finalize)
extern "C" int ffc_bn_reduce_finalize(const float* slab, int nrows, int C, double* moments, const float* gamma,
                                      const float* beta, float* running_mean, float* running_var,
                                      int64_t* num_batches_tracked, int update_running, float momentum, float eps,
                                      float count_mult, float* scale, float* shift, void* stream) {
    FFC_CHECK_ARG(slab && moments && nrows > 0 && C > 0 && scale && shift, "ffc_bn_reduce_finalize: bad args");
    FFC_CHECK_ARG(!update_running || (running_mean && running_var && num_batches_tracked),
                  "ffc_bn_reduce_finalize: update needs running buffers");
    FinalizeArgs a = make_finalize(gamma, beta, running_mean, running_var, num_batches_tracked, 1, update_running,
                                   momentum, eps, count_mult, scale, shift);
    if (red2_splits(nrows, C))
        bn_reduce2(slab, nrows, C, moments, &a, (hipStream_t)stream);
    else
        hipLaunchKernelGGL(bn_reduce_finalize_kernel, dim3(C), dim3(RED_THREADS), 0, (hipStream_t)stream,
                           reinterpret_cast<const float4*>(slab), nrows, C, moments, a);
    if (update_running && !a.bump_here)
        hipLaunchKernelGGL(bn_bump_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, num_batches_tracked);
    return ffc::launch_status("ffc_bn_reduce_finalize");
}

extern "C" int ffc_bn_act_apply(const float* x, float* y, int B, int C, int HW, const float* scale,
                                const float* shift, int act, float act_param, void* stream) {
    FFC_CHECK_ARG(x && y && scale && shift && B > 0 && C > 0 && HW > 0, "ffc_bn_act_apply: bad args");
    const long long total = (long long)B * C * HW;
    const bool vec = (total % 4 == 0) && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) % 16 == 0);
    if (vec && HW % 4 == 0 && HW >= 256) {
        const int HW4 = HW / 4, chunks = (HW4 + PLANE_CHUNK4 - 1) / PLANE_CHUNK4;
        hipLaunchKernelGGL(bn_act_plane_kernel, dim3((unsigned)(B * C * chunks)), dim3(256), 0, (hipStream_t)stream,
                           reinterpret_cast<const float4*>(x), reinterpret_cast<float4*>(y), C, HW4, chunks, scale,
                           shift, act, act_param, nullptr, nullptr);
    } else if (vec) {
        const long long t4 = total / 4;
        const int grid = (int)std::min<long long>((t4 + 255) / 256, 2048);
        hipLaunchKernelGGL(bn_act_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, y, C, HW, t4, scale,
                           shift, act, act_param);
    } else {
        const int grid = (int)std::min<long long>((total + 255) / 256, 2048);
        hipLaunchKernelGGL(bn_act_scalar_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, y, C, HW, total,
                           scale, shift, act, act_param);
    }
    return ffc::launch_status("ffc_bn_act_apply");
}

extern "C" int ffc_se_gate(const float* x, int B, int C, int H, int W, int pool, const float* w1, const float* w2,
                           int hidden, float* gate, void* stream) {
    FFC_CHECK_ARG(x && gate && B > 0 && C > 0 && H > 0 && W > 0 && hidden >= 0, "ffc_se_gate: bad args");
    FFC_CHECK_ARG(hidden == 0 || (w1 && w2), "ffc_se_gate: null weights");
    const size_t lds = sizeof(float) * (C + hidden);
    const bool wide = (W % 4 == 0) && (!pool || (H % 2 == 0 && W % 2 == 0)) && H * W >= 64 &&
                      (reinterpret_cast<uintptr_t>(x) & 15) == 0;
    if (wide) {
        // plane means into the gate buffer, then the FCs in place (each sample's block reads its
        // C means into LDS before any gate is written)
        const int planes = B * C;
        hipLaunchKernelGGL(se_mean_kernel, dim3((planes + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                           reinterpret_cast<const float4*>(x), planes, H * W / 4, 1.0f / (float)(H * W), gate);
        hipLaunchKernelGGL(se_fc_kernel, dim3(B), dim3(256), lds, (hipStream_t)stream, gate, C, w1, w2, hidden, gate);
    } else {
        hipLaunchKernelGGL(se_gate_kernel, dim3(B), dim3(256), lds, (hipStream_t)stream, x, C, H, W, pool, w1, w2,
                           hidden, gate);
    }
    return ffc::launch_status("ffc_se_gate");
}

extern "C" int ffc_bn_act_noise_apply(const float* x, float* y, int B, int C, int HW, const float* scale,
                                      const float* shift, int act, float act_param, const float* noise_w,
                                      const float* noise, void* stream) {
    FFC_CHECK_ARG(x && y && scale && shift && noise_w && noise && B > 0 && C > 0 && HW > 0,
                  "ffc_bn_act_noise_apply: bad args");
    FFC_CHECK_ARG(HW % 4 == 0 && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) |
                                   reinterpret_cast<uintptr_t>(noise)) & 15) == 0,
                  "ffc_bn_act_noise_apply: H*W % 4 == 0 and 16-byte aligned tensors required");
    const int HW4 = HW / 4, chunks = (HW4 + PLANE_CHUNK4 - 1) / PLANE_CHUNK4;
    hipLaunchKernelGGL(bn_act_plane_kernel, dim3((unsigned)(B * C * chunks)), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const float4*>(x), reinterpret_cast<float4*>(y), C, HW4, chunks, scale, shift,
                       act, act_param, noise_w, reinterpret_cast<const float4*>(noise));
    return ffc::launch_status("ffc_bn_act_noise_apply");
}

extern "C" int ffc_bn_reduce_finalize_batch(const ffc_bn_rf_item* items, int n, void* stream) {
    FFC_CHECK_ARG(items && n >= 1 && n <= FFC_MAX_BN_BATCH, "ffc_bn_reduce_finalize_batch: 1 <= n <= 4 items");
    RfBatch a = {};
    int blocks = 0;
    for (int i = 0; i < n; ++i) {
        const ffc_bn_rf_item& t = items[i];
        FFC_CHECK_ARG(t.slab && t.moments && t.nrows > 0 && t.C > 0 && t.scale && t.shift,
                      "ffc_bn_reduce_finalize_batch: bad item");
        FFC_CHECK_ARG(!t.update_running || (t.running_mean && t.running_var && t.num_batches_tracked),
                      "ffc_bn_reduce_finalize_batch: update needs running buffers");
    }
    for (int i = 0; i < n; ++i) {
        const ffc_bn_rf_item& t = items[i];
        if (red2_splits(t.nrows, t.C)) {   // large slab: its own two-level launches
            const int rc = ffc_bn_reduce_finalize(t.slab, t.nrows, t.C, t.moments, t.gamma, t.beta, t.running_mean,
                                                  t.running_var, t.num_batches_tracked, t.update_running, t.momentum,
                                                  t.eps, t.count_mult, t.scale, t.shift, stream);
            if (rc) return rc;
            continue;
        }
        const int k = a.n++;
        a.slab[k] = reinterpret_cast<const float4*>(t.slab);
        a.moments[k] = t.moments;
        a.fa[k] = make_finalize(t.gamma, t.beta, t.running_mean, t.running_var, t.num_batches_tracked, 1,
                                t.update_running, t.momentum, t.eps, t.count_mult, t.scale, t.shift);
        a.nrows[k] = t.nrows;
        a.C[k] = t.C;
        a.off[k] = blocks;
        blocks += t.C;
    }
    if (a.n == 0) return FFC_OK;
    a.off[a.n] = blocks;
    hipLaunchKernelGGL(bn_reduce_finalize_batch_kernel, dim3(blocks), dim3(RED_THREADS), 0, (hipStream_t)stream, a);
    for (int k = 0; k < a.n; ++k)   // momentum=None reads num_batches_tracked in every block: bump after
        if (a.fa[k].update_running && !a.fa[k].bump_here)
            hipLaunchKernelGGL(bn_bump_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, a.fa[k].nbt);
    return ffc::launch_status("ffc_bn_reduce_finalize_batch");
}

extern "C" int ffc_bn_act_apply_batch(const ffc_bn_apply_item* items, int n, void* stream) {
    FFC_CHECK_ARG(items && n >= 1 && n <= FFC_MAX_BN_BATCH, "ffc_bn_act_apply_batch: 1 <= n <= 4 items");
    ApplyBatch a = {};
    long long blocks = 0;
    for (int i = 0; i < n; ++i) {
        const ffc_bn_apply_item& t = items[i];
        FFC_CHECK_ARG(t.x && t.y && t.scale && t.shift && t.B > 0 && t.C > 0 && t.HW > 0,
                      "ffc_bn_act_apply_batch: bad item");
        FFC_CHECK_ARG(!t.noise || t.noise_w, "ffc_bn_act_apply_batch: noise needs noise_w");
        const bool plane = t.HW % 4 == 0 && t.HW >= 256 &&
                           ((reinterpret_cast<uintptr_t>(t.x) | reinterpret_cast<uintptr_t>(t.y) |
                             reinterpret_cast<uintptr_t>(t.noise)) & 15) == 0;
        FFC_CHECK_ARG(plane || !t.plane_sum, "ffc_bn_act_apply_batch: plane_sum needs HW % 4 == 0, HW >= 256, aligned");
        if (!plane) {   // the single forms' other paths
            const int rc = t.noise ? ffc_bn_act_noise_apply(t.x, t.y, t.B, t.C, t.HW, t.scale, t.shift, t.act,
                                                            t.act_param, t.noise_w, t.noise, stream)
                                   : ffc_bn_act_apply(t.x, t.y, t.B, t.C, t.HW, t.scale, t.shift, t.act, t.act_param,
                                                      stream);
            if (rc) return rc;
            continue;
        }
        const int k = a.n++;
        a.x[k] = reinterpret_cast<const float4*>(t.x);
        a.y[k] = reinterpret_cast<float4*>(t.y);
        a.scale[k] = t.scale;
        a.shift[k] = t.shift;
        a.noise_w[k] = t.noise ? t.noise_w : nullptr;
        a.noise[k] = reinterpret_cast<const float4*>(t.noise);
        a.psum[k] = t.plane_sum;
        a.C[k] = t.C;
        a.HW4[k] = t.HW / 4;
        a.chunks[k] = (t.HW / 4 + PLANE_CHUNK4 - 1) / PLANE_CHUNK4;
        a.act[k] = t.act;
        a.p[k] = t.act_param;
        a.off[k] = (int)blocks;
        blocks += (long long)t.B * t.C * a.chunks[k];
        FFC_CHECK_ARG(blocks < (1LL << 31), "ffc_bn_act_apply_batch: grid too large");
    }
    if (a.n == 0) return FFC_OK;
    a.off[a.n] = (int)blocks;
    hipLaunchKernelGGL(bn_act_plane_batch_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a);
    return ffc::launch_status("ffc_bn_act_apply_batch");
}

extern "C" int ffc_plane_chunks(int HW) { return HW > 0 ? (HW / 4 + PLANE_CHUNK4 - 1) / PLANE_CHUNK4 : 0; }

extern "C" int ffc_se_gate_sums(const float* sums, int chunks, int B, int C, int HW, const float* w1, const float* w2,
                                int hidden, float* gate, void* stream) {
    FFC_CHECK_ARG(sums && gate && B > 0 && C > 0 && HW > 0 && hidden >= 0 && chunks == ffc_plane_chunks(HW),
                  "ffc_se_gate_sums: bad args");
    FFC_CHECK_ARG(hidden == 0 || (w1 && w2), "ffc_se_gate_sums: null weights");
    hipLaunchKernelGGL(se_fc_sums_kernel, dim3(B), dim3(256), sizeof(float) * (C + hidden), (hipStream_t)stream, sums,
                       chunks, C, 1.0f / (float)HW, w1, w2, hidden, gate);
    return ffc::launch_status("ffc_se_gate_sums");
}
