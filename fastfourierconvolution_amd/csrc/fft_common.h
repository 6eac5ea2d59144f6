// Register-resident radix-2 FFT and the twiddle table shared by the Fourier-unit kernels
// (fu_kernels.hip: fused per-sample FU; fu2d_kernels.hip: large-plane FU stages).
#pragma once
#include "ffc_internal.h"

namespace {

#include "twiddles.inc"

// Lanes of ONE wave exchanging values through LDS (the line FFTs' stage B, the r2c half-spectrum
// separation, the c2r row hand-off): a lane reads slots other lanes of its wave wrote, or overwrites
// slots they still read.  The hardware keeps a wave's LDS operations in issue order, but the
// compiler reasons per lane: with no synchronisation between the lanes the exchange is a data race
// in the HIP memory model, and the compiler may move a lane's load past its own store to a slot it
// believes unrelated (or the reverse).  The r03 -fno-slp-vectorize build did exactly that in
// fu2d_kernels.hip: correct results depended on the vectorizer.  A wavefront-scope
// release / acquire fence pair around wave_barrier orders the LDS accesses across the exchange for
// the compiler; at wavefront scope the fences emit no instruction (AMDGPU memory model), so the
// order costs nothing at run time.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr int ilog2c(int n) { return n <= 1 ? 0 : 1 + ilog2c(n >> 1); }
constexpr int brevc(int i, int bits) {
    int r = 0;
    for (int b = 0; b < bits; ++b) r |= ((i >> b) & 1) << (bits - 1 - b);
    return r;
}

// In-register radix-2 DIT FFT, fully unrolled.  INV=false: exp(-2 pi i kn/N); INV=true: exp(+..).
// N <= 128 (twiddles from the 128-entry table).
template <int N, bool INV>
__device__ __forceinline__ void fft_reg(float (&re)[N], float (&im)[N]) {
    constexpr int L = ilog2c(N);
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const int j = brevc(i, L);
        if (j > i) {
            float t = re[i]; re[i] = re[j]; re[j] = t;
            t = im[i]; im[i] = im[j]; im[j] = t;
        }
    }
#pragma unroll
    for (int half = 1; half < N; half <<= 1) {
        const int step = 128 / (2 * half);
#pragma unroll
        for (int j = 0; j < half; ++j) {
            // twiddle W_{2 half}^j: 1 at j = 0, -i (forward) / +i (inverse) at the quarter turn -- both
            // multiply-free (the table's cos(pi/2) is 6e-17, not 0); the rest from the table
            const bool quarter = j * step == 32;
            float wr = 1.0f, wi = 0.0f;
            if (j != 0) {
                wr = c_twc[j * step];
                wi = INV ? c_tws[j * step] : -c_tws[j * step];
            }
#pragma unroll
            for (int i = j; i < N; i += 2 * half) {
                float xr, xi;
                if (j == 0) {
                    xr = re[i + half];
                    xi = im[i + half];
                } else if (quarter) {
                    xr = INV ? -im[i + half] : im[i + half];
                    xi = INV ? re[i + half] : -re[i + half];
                } else {
                    xr = re[i + half] * wr - im[i + half] * wi;
                    xi = re[i + half] * wi + im[i + half] * wr;
                }
                re[i + half] = re[i] - xr;
                im[i + half] = im[i] - xi;
                re[i] += xr;
                im[i] += xi;
            }
        }
    }
}

// Real-input N-point DFT X[k] = sum_n x[n] exp(-2 pi i k n / N), k = 0 .. N/2, through ONE
// N/2-point complex FFT of z[n] = x[2n] + i x[2n+1] (half the butterflies and registers of
// fft_reg<N> on (x, 0)):  X[k] = E[k] + W^k O[k],  E = (Z[k] + conj Z[M-k]) / 2,
// O = (Z[k] - conj Z[M-k]) / 2i,  W = exp(-2 pi i / N),  M = N/2 (Z[M] = Z[0]).
template <int N>
__device__ __forceinline__ void rfft_reg(const float (&x)[N], float (&Xr)[N / 2 + 1], float (&Xi)[N / 2 + 1]) {
    constexpr int M = N / 2;
    float zr[M], zi[M];
#pragma unroll
    for (int n = 0; n < M; ++n) {
        zr[n] = x[2 * n];
        zi[n] = x[2 * n + 1];
    }
    fft_reg<M, false>(zr, zi);
    Xr[0] = zr[0] + zi[0];
    Xi[0] = 0.0f;
    Xr[M] = zr[0] - zi[0];
    Xi[M] = 0.0f;
#pragma unroll
    for (int k = 1; k < M; ++k) {
        const float ar = zr[k], ai = zi[k], br = zr[M - k], bi = zi[M - k];
        const float er = 0.5f * (ar + br), ei = 0.5f * (ai - bi);
        const float orr = 0.5f * (ai + bi), oi = 0.5f * (br - ar);
        if (4 * k == N) {   // W^k = -i
            Xr[k] = er + oi;
            Xi[k] = ei - orr;
        } else {
            const float c = c_twc[k * (128 / N)], s = c_tws[k * (128 / N)];   // W^k = c - i s
            Xr[k] = er + (orr * c + oi * s);
            Xi[k] = ei + (oi * c - orr * s);
        }
    }
}

// Its inverse without normalisation, the C2R of irfftn: x[n] = sum_{k<N} F[k] exp(+2 pi i k n / N)
// with F[k] = X[k] (k <= N/2, Im of X[0] and X[N/2] ignored) and F[N-k] = conj X[k], through ONE
// N/2-point inverse FFT of Z[k] = (F[k] + F[k+M]) + i W^-k (F[k] - F[k+M]) (F[k+M] = conj X[M-k]):
// z[n] = x[2n] + i x[2n+1].
template <int N>
__device__ __forceinline__ void irfft_reg(const float (&Xr)[N / 2 + 1], const float (&Xi)[N / 2 + 1], float (&x)[N]) {
    constexpr int M = N / 2;
    float zr[M], zi[M];
    zr[0] = Xr[0] + Xr[M];
    zi[0] = Xr[0] - Xr[M];
#pragma unroll
    for (int k = 1; k < M; ++k) {
        const float ar = Xr[k], ai = Xi[k], br = Xr[M - k], bi = Xi[M - k];
        const float sr = ar + br, si = ai - bi;   // F[k] + conj X[M-k]
        const float dr = ar - br, di = ai + bi;   // F[k] - conj X[M-k]
        float tr, ti;                             // T = W^-k D, W^-k = c + i s
        if (4 * k == N) {
            tr = -di;
            ti = dr;
        } else {
            const float c = c_twc[k * (128 / N)], s = c_tws[k * (128 / N)];
            tr = dr * c - di * s;
            ti = dr * s + di * c;
        }
        zr[k] = sr - ti;   // Z = S + i T
        zi[k] = si + tr;
    }
    fft_reg<M, true>(zr, zi);
#pragma unroll
    for (int n = 0; n < M; ++n) {
        x[2 * n] = zr[n];
        x[2 * n + 1] = zi[n];
    }
}

// ---- Column DFTs across lanes (wave-64 butterfly exchanges, round 6)
// The fused Fourier unit holds one spectrum row per lane after its row R2C (fu_kernels.hip: lane
// y of an aligned group of N lanes = row y of one channel, re[k] / im[k] = bin k of that row).
// The column DFT of bin k then runs ACROSS the group's lanes: a radix-2 butterfly pairs lane y with
// lane y ^ D, and the partner's value comes through a lane exchange instead of an LDS write /
// barrier / strided read / write round trip:
//   D = 1, 2   one DPP quad_perm move,
//   D = 4      row_half_mirror (y ^ 7) then quad_perm [3,2,1,0] (^ 3),
//   D = 8      row_mirror (y ^ 15) then row_half_mirror (^ 7),
//   D = 16     ds_swizzle in bit-mask mode (xor 16 within 32 lanes; no LDS memory access).
// Both lanes of a pair compute one output each, branch-free: t = p + sg v with sg = +1 on the
// lower lane (a + b) and -1 on the upper (a - b), then the upper lane's twiddle.
// Measured on MI355X (gen64 B = 256, same-box A/B): the DPP composites cost VALU issue
// and wait states in a VALU-bound phase; ds_swizzle for every distance (the exchange on the LDS
// pipe, no memory access) with packed (re, im) arithmetic is the fastest form (FFC_LANE_SWZ = 2,
// FFC_LANE_PK), level with the LDS column pass, which stays the default (FFC_FU_SHUF=1 selects this).
#ifndef FFC_LANE_NOPK
#define FFC_LANE_PK
#endif
template <int D>
__device__ __forceinline__ float lane_xor(float v) {
    static_assert(D == 1 || D == 2 || D == 4 || D == 8 || D == 16, "partner distance within 32 lanes");
    const int iv = __builtin_bit_cast(int, v);
    int r;
#ifndef FFC_LANE_SWZ
#define FFC_LANE_SWZ 2   // 2: ds_swizzle for every D; 1: for D >= 4; 0: the DPP moves above (A/B)
#endif
    if constexpr (FFC_LANE_SWZ == 2 || (FFC_LANE_SWZ == 1 && D >= 4)) {
        r = __builtin_amdgcn_ds_swizzle(iv, (D << 10) | 0x1F);
    } else if constexpr (D == 1) {
        r = __builtin_amdgcn_update_dpp(0, iv, 0xB1, 0xF, 0xF, false);
    } else if constexpr (D == 2) {
        r = __builtin_amdgcn_update_dpp(0, iv, 0x4E, 0xF, 0xF, false);
    } else if constexpr (D == 4) {
        r = __builtin_amdgcn_update_dpp(0, __builtin_amdgcn_update_dpp(0, iv, 0x141, 0xF, 0xF, false), 0x1B, 0xF,
                                        0xF, false);
    } else if constexpr (D == 8) {
        r = __builtin_amdgcn_update_dpp(0, __builtin_amdgcn_update_dpp(0, iv, 0x140, 0xF, 0xF, false), 0x141, 0xF,
                                        0xF, false);
    } else {
        r = __builtin_amdgcn_ds_swizzle(iv, 0x401F);   // and_mask 0x1F, or_mask 0, xor_mask 16
    }
    return __builtin_bit_cast(float, r);
}

// row index bitrev(y) over log2(N) bits (the DIF output order)
template <int N>
__device__ __forceinline__ int lane_brev(int y) {
    return (int)(__builtin_bitreverse32((unsigned)y) >> (32 - ilog2c(N)));
}

// twiddle of lane y at the stage of half-size D (sub-transforms of length 2D): W_{2D}^{y mod D} on the
// upper lane of the pair (y & D), 1 on the lower.  Forward exp(-2 pi i j / 2D), INV exp(+..)
template <int D, bool INV>
__device__ __forceinline__ void lane_tw(int y, float& c, float& s) {
    const int j = y & (D - 1);
    const bool up = (y & D) != 0;
    const float tc = c_twc[j * (64 / D)], ts = c_tws[j * (64 / D)];
    c = up ? tc : 1.0f;
    s = up ? (INV ? ts : -ts) : 0.0f;
}

// decimation-in-frequency stage D: exchange, add / subtract, twiddle (D = 1: the factor `scale`)
template <int D, int K>
__device__ __forceinline__ void lane_dif_stage(float (&re)[K], float (&im)[K], int y, float scale) {
    const float sg = (y & D) ? -1.0f : 1.0f;
    float c, s;
    lane_tw<D, false>(y, c, s);
#ifdef FFC_LANE_PK   // the add / subtract and the twiddle on packed (re, im) pairs (FFC_LANE_NOPK: scalar)
    typedef float lf2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const lf2 v = {re[k], im[k]};
        const lf2 p = {lane_xor<D>(re[k]), lane_xor<D>(im[k])};
        const lf2 t = __builtin_elementwise_fma(lf2{sg, sg}, v, p);
        lf2 o;
        if constexpr (D == 1) {
            o = t * scale;
        } else {
            o = __builtin_elementwise_fma(lf2{t.y, t.x}, lf2{-s, s}, t * c);
        }
        re[k] = o.x;
        im[k] = o.y;
    }
    return;
#endif
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const float pr = lane_xor<D>(re[k]), pi = lane_xor<D>(im[k]);
        const float tr = fmaf(sg, re[k], pr), ti = fmaf(sg, im[k], pi);
        if constexpr (D == 1) {
            re[k] = tr * scale;
            im[k] = ti * scale;
        } else {
            re[k] = fmaf(tr, c, -ti * s);
            im[k] = fmaf(tr, s, ti * c);
        }
    }
}

// decimation-in-time inverse stage D: twiddle (D = 1: the factor `scale` on both lanes), exchange,
// add / subtract
template <int D, int K>
__device__ __forceinline__ void lane_dit_inv_stage(float (&re)[K], float (&im)[K], int y, float scale) {
    const float sg = (y & D) ? -1.0f : 1.0f;
    float c, s;
    lane_tw<D, true>(y, c, s);
#ifdef FFC_LANE_PK
    typedef float lf2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const lf2 v = {re[k], im[k]};
        lf2 u;
        if constexpr (D == 1) {
            u = v * scale;
        } else {
            u = __builtin_elementwise_fma(lf2{v.y, v.x}, lf2{-s, s}, v * c);
        }
        const lf2 p = {lane_xor<D>(u.x), lane_xor<D>(u.y)};
        const lf2 o = __builtin_elementwise_fma(lf2{sg, sg}, u, p);
        re[k] = o.x;
        im[k] = o.y;
    }
    return;
#endif
#pragma unroll
    for (int k = 0; k < K; ++k) {
        float ur, ui;
        if constexpr (D == 1) {
            ur = re[k] * scale;
            ui = im[k] * scale;
        } else {
            ur = fmaf(re[k], c, -im[k] * s);
            ui = fmaf(re[k], s, im[k] * c);
        }
        const float pr = lane_xor<D>(ur), pi = lane_xor<D>(ui);
        re[k] = fmaf(sg, ur, pr);
        im[k] = fmaf(sg, ui, pi);
    }
}

// Forward N-point DFT over the N lanes of an aligned lane group, K columns at once: lane y holds x[y]
// (per column) and ends with scale * X[bitrev(y)].  Every lane of the group must be active.
template <int N, int K>
__device__ __forceinline__ void lane_fft_dif(float (&re)[K], float (&im)[K], int y, float scale) {
    static_assert(N >= 2 && N <= 32 && (N & (N - 1)) == 0, "2 .. 32 lanes");
    if constexpr (N > 16) lane_dif_stage<16, K>(re, im, y, scale);
    if constexpr (N > 8) lane_dif_stage<8, K>(re, im, y, scale);
    if constexpr (N > 4) lane_dif_stage<4, K>(re, im, y, scale);
    if constexpr (N > 2) lane_dif_stage<2, K>(re, im, y, scale);
    lane_dif_stage<1, K>(re, im, y, scale);
}

// Inverse (unnormalised, times `scale`) N-point DFT over the lane group: lane y holds X[bitrev(y)]
// and ends with scale * x[y], x[n] = sum_k X[k] exp(+2 pi i k n / N).
template <int N, int K>
__device__ __forceinline__ void lane_ifft_dit(float (&re)[K], float (&im)[K], int y, float scale) {
    static_assert(N >= 2 && N <= 32 && (N & (N - 1)) == 0, "2 .. 32 lanes");
    lane_dit_inv_stage<1, K>(re, im, y, scale);
    if constexpr (N > 2) lane_dit_inv_stage<2, K>(re, im, y, scale);
    if constexpr (N > 4) lane_dit_inv_stage<4, K>(re, im, y, scale);
    if constexpr (N > 8) lane_dit_inv_stage<8, K>(re, im, y, scale);
    if constexpr (N > 16) lane_dit_inv_stage<16, K>(re, im, y, scale);
}

}  // namespace
