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

}  // namespace
