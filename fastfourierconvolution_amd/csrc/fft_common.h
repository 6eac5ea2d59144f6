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

}  // namespace
