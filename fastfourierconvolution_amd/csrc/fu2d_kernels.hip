// Large-plane Fourier unit for gfx950 (FU planes that do not fit one workgroup's LDS per sample:
// the fgan128 generator's 64x64 and 128x128 FUs, fgan128_complete.py:474-485).
//
// Replaces FourierUnitSN.forward (layers/ffc/fourier_unity.py:32-56) with three HBM stages:
//
//   r2c  one workgroup per (sample, channel) plane of t (h x w = H/up x W/up):
//        s0 = relu(t*in_scale + in_shift) (bn1 + act1, spectral_transform.py:89), 2-D real FFT
//        in LDS -> T (B, C, h, w/2+1) complex, unnormalised.
//   mix  per (sample, bin range): rebuild X = rfftn(s, ortho) from T, where s is s0
//        nearest-upsampled by `up` (spectral_transform.py:44-45), using the identity
//            X[kh][kw] = T[kh mod h][kw mod w] (1 + e^{-2 pi i kh/H}) (1 + e^{-2 pi i kw/W}) / sqrt(HW)
//        (T folded through Hermitian symmetry for kw mod w > w/2), then the 1x1 spectral mix
//        Y = Wmix Z on v_mfma_f32_32x32x2_f32 (Z = the interleaved Re/Im channels, :40-45).
//        pass 0: BatchNorm partials {n, mean, M2} per output channel -> one slab row per workgroup
//        pass 1: relu(Y*bn_scale + bn_shift) (:46-49) -> Y (B, C, H, W/2+1) complex
//   c2r  one workgroup per output plane: irfftn(Y, s=(H, W), ortho) (:51-56) -- inverse column
//        FFT, then the row C2R that ignores Im of bins 0 and W/2 (torch's C2R semantics) -- plus
//        the SpectralTransform residual s (spectral_transform.py:108) -> out (B, C, H, W).
//
// Line FFTs of length N = N1*N2 are split over the N1 lanes of one wave: each lane runs an
// N2-point FFT in registers, multiplies the twiddles W_N^{j k2}, and the lanes exchange through
// the line's own LDS slots for the N1-point FFTs (same wave: no workgroup barrier; every exchange
// is fenced for the compiler by wave_lds_sync, fft_common.h).  The upsample identity lets r2c
// transform the 4x smaller t plane, and the mix reads the 4x smaller T, so HBM carries: r2c t + T,
// mix T (+ Y), c2r Y + t + out.
#include "ffc_internal.h"

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <mutex>
#include <set>

#include "fft_common.h"
#include "bn_common.h"

namespace {

constexpr int FU2_THREADS = 256;

template <int N>
struct Split {
    static constexpr int N1 = N >= 64 ? 8 : (N >= 16 ? 4 : 2);
    static constexpr int N2 = N / N1;
    static constexpr int Q = N2 / N1;
    static_assert(N1 * N2 == N && N2 % N1 == 0 && N <= 128, "line FFT split");
};

// twiddle W_N^e (e in [0, N)), forward exp(-2 pi i e/N) or inverse exp(+..)
template <int N, bool INV>
__device__ __forceinline__ void twiddle(int e, float& c, float& s) {
    c = c_twc[e * (128 / N)];
    s = INV ? c_tws[e * (128 / N)] : -c_tws[e * (128 / N)];
}

// This lane's stage-A twiddles W_N^{jj*k2} (k2 = 1..N2-1; jj*k2 < N): loaded once per kernel, before
// its line loops -- inside them every line FFT paid a dependent table load (per-lane index, so a
// vector-memory load) before its twiddle multiplies.
template <int N>
struct LaneTw {
    float c[Split<N>::N2], s[Split<N>::N2];
    __device__ __forceinline__ explicit LaneTw(int jj) {
#pragma unroll
        for (int k2 = 1; k2 < Split<N>::N2; ++k2) {
            c[k2] = c_twc[jj * k2 * (128 / N)];
            s[k2] = c_tws[jj * k2 * (128 / N)];
        }
    }
};

// Stage A on this lane's samples x[jj + N1*m] (m = 0..N2-1, in re/im): N2-point FFT in registers,
// then the twiddles W_N^{jj*k2}.  Result index k2 holds Y[jj][k2].
template <int N, bool INV>
__device__ __forceinline__ void stage_a(float (&re)[Split<N>::N2], float (&im)[Split<N>::N2], const LaneTw<N>& tw) {
    constexpr int N2 = Split<N>::N2;
    fft_reg<N2, INV>(re, im);
#pragma unroll
    for (int k2 = 1; k2 < N2; ++k2) {
        const float c = tw.c[k2], s = INV ? tw.s[k2] : -tw.s[k2];
        const float xr = re[k2] * c - im[k2] * s;
        im[k2] = re[k2] * s + im[k2] * c;
        re[k2] = xr;
    }
}
template <int N, bool INV>
__device__ __forceinline__ void stage_a(float (&re)[Split<N>::N2], float (&im)[Split<N>::N2], int jj) {
    stage_a<N, INV>(re, im, LaneTw<N>(jj));
}

// Stage B through an LDS line of N float2 (element n at line[n*stride]): writes stage-A results,
// reads back the N1-point columns k2 in {jj, jj+N1, ..} and transforms them.  On return
// (ore, oim)[q][k1] = X[(jj + N1*q) + N2*k1].  Every lane of the group must call it (one wave).
template <int N, bool INV>
__device__ __forceinline__ void stage_b(float2* line, int stride, const float (&re)[Split<N>::N2],
                                        const float (&im)[Split<N>::N2], int jj,
                                        float (&ore)[Split<N>::Q][Split<N>::N1],
                                        float (&oim)[Split<N>::Q][Split<N>::N1]) {
    constexpr int N1 = Split<N>::N1, N2 = Split<N>::N2, Q = Split<N>::Q;
    wave_lds_sync();   // the group's earlier reads of this line precede these writes
#pragma unroll
    for (int k2 = 0; k2 < N2; ++k2) line[(jj + N1 * k2) * stride] = make_float2(re[k2], im[k2]);
    wave_lds_sync();   // every lane's stage-A results are in the line before anyone reads a column
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int k2 = jj + N1 * q;
#pragma unroll
        for (int n1 = 0; n1 < N1; ++n1) {
            const float2 v = line[(n1 + N1 * k2) * stride];
            ore[q][n1] = v.x;
            oim[q][n1] = v.y;
        }
    }
    wave_lds_sync();   // every lane's reads are done before a caller overwrites the line
#pragma unroll
    for (int q = 0; q < Q; ++q) fft_reg<N1, INV>(ore[q], oim[q]);
}

// In-place length-N complex FFT of line[n*stride] by the N1 lanes jj of one wave.
template <int N, bool INV>
__device__ __forceinline__ void line_fft(float2* line, int stride, int jj, const LaneTw<N>& tw) {
    constexpr int N1 = Split<N>::N1, N2 = Split<N>::N2, Q = Split<N>::Q;
    float re[N2], im[N2];
#pragma unroll
    for (int m = 0; m < N2; ++m) {
        const float2 v = line[(jj + N1 * m) * stride];
        re[m] = v.x;
        im[m] = v.y;
    }
    stage_a<N, INV>(re, im, tw);
    float ore[Q][N1], oim[Q][N1];
    stage_b<N, INV>(line, stride, re, im, jj, ore, oim);
#pragma unroll
    for (int q = 0; q < Q; ++q)
#pragma unroll
        for (int k1 = 0; k1 < N1; ++k1)
            line[((jj + N1 * q) + N2 * k1) * stride] = make_float2(ore[q][k1], oim[q][k1]);
}

// Column pass over an (rows x ZS) float2 plane: length-`rows` FFTs of columns 0..ncols-1.
template <int ROWS, bool INV, int NT = FU2_THREADS>
__device__ __forceinline__ void column_pass(float2* Z, int ZS, int ncols, int tid) {
    constexpr int N1 = Split<ROWS>::N1;
    constexpr int LPR = NT / N1;   // lines per round
    const int jj = tid % N1;
    const LaneTw<ROWS> tw(jj);
    for (int c0 = 0; c0 < ncols; c0 += LPR) {
        const int col = c0 + tid / N1;
        if (col < ncols) line_fft<ROWS, INV>(Z + col, ZS, jj, tw);
    }
}

// LDS row stride (float2) of a half-spectrum plane with WP = W/2+1 columns: WP rounded up to 4 mod 8,
// so the 8 lanes x 8 adjacent columns of a wave in the column pass (row stride * jj + column) and
// the 8 row pairs x 8 lanes of the row pass spread over the 64 banks (the unpadded odd stride put
// a wave on ~15 bank pairs).
constexpr int zstride(int WP) { return ((WP + 3) & ~7) + 4; }

__device__ __forceinline__ float in_tf(float v, float sc, float sh, int relu) {
    v = fmaf(v, sc, sh);
    return relu ? fmaxf(v, 0.0f) : v;
}

struct R2cArgs {
    const float* t;
    const float* in_scale;
    const float* in_shift;
    float* T;
    int C, in_relu;
    float oscale, iscale;   // PLANAR: every bin x oscale, bins with a Hermitian mirror x iscale too
    int has_fold;           // the input BN (SpectralTransform.bn1) finalized here, per plane channel
    ffc_bn_fold fold;       // (in_scale / in_shift unused; the channel leaders write scale_out / shift_out)
};

// ---------------------------------------------------------------- stage 1: R2C of the t planes
// LDS: real plane R (h rows, stride w+4: conflict-free row-pair reads), complex plane Z (h x WPt).
// PLANAR (the training path's ffc_rfft2_planes): T is the interleaved channel-plane layout of
// fourier_unity.py:40-42 -- Re of plane p at T + 2p*h*WPt, Im at T + (2p+1)*h*WPt -- scaled by
// oscale (1/sqrt(hw): rfftn ortho) and, on bins 0 < kw < w/2, iscale (2: the adjoint of irfftn).
template <int h, int w, bool PLANAR = false>
__global__ __launch_bounds__(FU2_THREADS) void fu2d_r2c_kernel(R2cArgs a) {
    constexpr int WPt = w / 2 + 1;
    constexpr int ZS = zstride(WPt);
    constexpr int RS = w + 4;
    constexpr int N1 = Split<w>::N1, N2 = Split<w>::N2, Q = Split<w>::Q;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* R = smem;
    float2* Z = reinterpret_cast<float2*>(smem + h * RS);
    const int plane = blockIdx.x;
    const int ch = plane % a.C;
    const int tid = threadIdx.x;
    float sc = a.in_scale ? a.in_scale[ch] : 1.0f;
    float sh = a.in_scale ? a.in_shift[ch] : 0.0f;

    // 1. t plane -> transform -> R
    const float4* src = reinterpret_cast<const float4*>(a.t + (size_t)plane * h * w);
    constexpr int NV = (h * w / 4 + FU2_THREADS - 1) / FU2_THREADS;   // float4 per thread, all in flight
    float4 v[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int i = j * FU2_THREADS + tid;
        if (i < h * w / 4) v[j] = src[i];
    }
    if (!PLANAR && a.has_fold) {
        // bn1 of this plane's channel from its slab rows, under the plane loads' latency; the
        // workgroups of sample 0 lead (running statistics, scale_out / shift_out for the C2R)
        float* fsc = smem + h * RS + 2 * h * ZS;   // 16 B behind the planes (r2c_lds; no static LDS:
                                                   // it would cap the dynamic size below 160 KiB)
        if (tid < 64) {
            float fs, fh;
            ffc::bn_fold_channel(a.fold, ch, plane < a.C, fs, fh);
            if (tid == 0) {
                fsc[0] = fs;
                fsc[1] = fh;
                if (plane == 0 && a.fold.update_running) *a.fold.num_batches_tracked += 1;
            }
        }
        __syncthreads();
        sc = fsc[0];
        sh = fsc[1];
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int i = j * FU2_THREADS + tid;
        if (i < h * w / 4) {
            float4 q = v[j];
            q.x = in_tf(q.x, sc, sh, a.in_relu);
            q.y = in_tf(q.y, sc, sh, a.in_relu);
            q.z = in_tf(q.z, sc, sh, a.in_relu);
            q.w = in_tf(q.w, sc, sh, a.in_relu);
            const int r = i / (w / 4), c4 = i % (w / 4);
            *reinterpret_cast<float4*>(R + r * RS + 4 * c4) = q;
        }
    }
    __syncthreads();

    // 2. rows, two at a time: z = R[2g] + i R[2g+1] -> FFT -> split into the two half spectra
    {
        constexpr int LPR = FU2_THREADS / N1;
        const int jj = tid % N1;
        const LaneTw<w> twr(jj);
        for (int g0 = 0; g0 < h / 2; g0 += LPR) {
            const int g = g0 + tid / N1;
            if (g < h / 2) {
                float re[N2], im[N2];
#pragma unroll
                for (int m = 0; m < N2; ++m) {
                    re[m] = R[(2 * g) * RS + jj + N1 * m];
                    im[m] = R[(2 * g + 1) * RS + jj + N1 * m];
                }
                stage_a<w, false>(re, im, twr);
                float2* line = Z + 2 * g * ZS;    // rows 2g, 2g+1 of Z: 2*ZS >= w slots
                float ore[Q][N1], oim[Q][N1];
                stage_b<w, false>(line, 1, re, im, jj, ore, oim);
#pragma unroll
                for (int q = 0; q < Q; ++q)
#pragma unroll
                    for (int k1 = 0; k1 < N1; ++k1)
                        line[(jj + N1 * q) + N2 * k1] = make_float2(ore[q][k1], oim[q][k1]);
                wave_lds_sync();   // the whole spectrum is in the line
                // separate: A[k] = (Z[k] + conj Z[-k]) / 2, B[k] = (Z[k] - conj Z[-k]) / 2i, k = 0..w/2
                constexpr int KPL = (WPt + N1 - 1) / N1;
                float2 zk[KPL], zm[KPL];
#pragma unroll
                for (int i = 0; i < KPL; ++i) {
                    const int k = jj + N1 * i;
                    if (k < WPt) {
                        zk[i] = line[k & (w - 1)];
                        zm[i] = line[(w - k) & (w - 1)];
                    }
                }
                wave_lds_sync();   // every lane has read Z[k] and Z[-k] before the halves overwrite them
#pragma unroll
                for (int i = 0; i < KPL; ++i) {
                    const int k = jj + N1 * i;
                    if (k < WPt) {
                        line[k] = make_float2(0.5f * (zk[i].x + zm[i].x), 0.5f * (zk[i].y - zm[i].y));
                        line[ZS + k] = make_float2(0.5f * (zk[i].y + zm[i].y), -0.5f * (zk[i].x - zm[i].x));
                    }
                }
            }
        }
    }
    __syncthreads();

    // 3. columns (length h) of the half spectrum
    column_pass<h, false>(Z, ZS, WPt, tid);
    __syncthreads();

    // 4. Z -> T (contiguous h x WPt float2, or the two planes of PLANAR)
    if constexpr (PLANAR) {
        float* re = a.T + (size_t)plane * 2 * h * WPt;
        float* im = re + h * WPt;
        for (int i = tid; i < h * WPt; i += FU2_THREADS) {
            const int r = i / WPt, k = i - r * WPt;
            const float sc = (k == 0 || 2 * k == w) ? a.oscale : a.oscale * a.iscale;
            const float2 v = Z[r * ZS + k];
            re[i] = v.x * sc;
            im[i] = v.y * sc;
        }
    } else {
        float2* dst = reinterpret_cast<float2*>(a.T) + (size_t)plane * h * WPt;
        for (int i = tid; i < h * WPt; i += FU2_THREADS) {
            const int r = i / WPt, k = i - r * WPt;
            dst[i] = Z[r * ZS + k];
        }
    }
}

// ---------------------------------------------------------------- stage 3: C2R + residual
struct C2rArgs {
    const float* Y;
    const float* t;
    const float* in_scale;
    const float* in_shift;
    float* out;
    int C, in_relu, residual;
    float norm;
    const float* bn_scale;   // optional [2C]: Y is the raw mix output, relu(Y*bn_scale + bn_shift) on load
    const float* bn_shift;
    float iscale;            // PLANAR: bins 0 < kw < W/2 x iscale (0.5: the adjoint of rfftn)
    int has_bn_fold;         // the FU's BN finalized here (channels 2c, 2c+1 of this plane) instead of
    ffc_bn_fold bn_fold;     // bn_scale / bn_shift; sample 0's workgroups lead
};

// PLANAR (the training path's ffc_irfft2_planes): Y in the interleaved channel-plane layout (Re of
// plane p at Y + 2p*H*WP, Im at Y + (2p+1)*H*WP), interior bins x iscale; UP = 1, residual = addend.
template <int H, int W, int UP, bool PLANAR = false>
__global__ __launch_bounds__(FU2_THREADS) void fu2d_c2r_kernel(C2rArgs a) {
    constexpr int WP = W / 2 + 1;
    constexpr int ZS = zstride(WP);
    constexpr int N1 = Split<W>::N1, N2 = Split<W>::N2, Q = Split<W>::Q;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float2* Z = reinterpret_cast<float2*>(smem);
    const int plane = blockIdx.x;
    const int ch = plane % a.C;
    const int tid = threadIdx.x;
    const LaneTw<H> twc(tid % Split<H>::N1);   // column IFFTs (step 2)
    const LaneTw<W> twr(tid % N1);             // row C2R (step 3)

    // 1. Y plane -> LDS rows of stride ZS; a raw (spilled) Y gets the FU's BN + ReLU here, the same
    //    expression as mix pass 1.  Non-planar: the whole plane as 16-byte loads (two complex bins,
    //    possibly across a row end), all issued before the first wait, and (UP = 2) the residual
    //    t values this thread adds in step 3 issued with them -- one memory latency per plane
    //    instead of three (two Y batches, then the residual under the row pass).
    const float sc = a.in_scale ? a.in_scale[ch] : 1.0f;
    const float sh = a.in_scale ? a.in_shift[ch] : 0.0f;
    constexpr int tW = W / UP;
    const float* tpl = a.t + (size_t)plane * (H / UP) * tW;
    float* opl = a.out + (size_t)plane * H * W;
    constexpr int RLPR = FU2_THREADS / N1;                      // row pairs per round of step 3
    constexpr int RROUNDS = (H / 2 + RLPR - 1) / RLPR;
    constexpr int RITER = (2 * W / 4 + N1 - 1) / N1;            // float4 outputs per thread per row pair
    constexpr bool RPRE = !PLANAR && UP == 2;
    float2 res[RPRE ? RROUNDS : 1][RPRE ? RITER : 1];
    {
        const bool bn = a.bn_scale != nullptr || a.has_bn_fold;
        float bsr = bn && !a.has_bn_fold ? a.bn_scale[2 * ch] : 1.0f, bhr = bn && !a.has_bn_fold ? a.bn_shift[2 * ch] : 0.0f;
        float bsi = bn && !a.has_bn_fold ? a.bn_scale[2 * ch + 1] : 1.0f;
        float bhi = bn && !a.has_bn_fold ? a.bn_shift[2 * ch + 1] : 0.0f;
        if constexpr (!PLANAR) {
            constexpr int N4 = H * WP / 2;                         // H even: whole float4 pairs
            constexpr int NL = (N4 + FU2_THREADS - 1) / FU2_THREADS;
            const float4* src4 = reinterpret_cast<const float4*>(a.Y) + (size_t)plane * N4;
            float4 v[NL];
#pragma unroll
            for (int u = 0; u < NL; ++u) {
                const int i = u * FU2_THREADS + tid;
                v[u] = src4[i < N4 ? i : 0];
            }
            if (a.has_bn_fold) {
                // the FU's BN of this plane's two spectral channels (Re 2c, Im 2c+1) from pass 0's slab
                // rows, waves 0 and 1 in parallel, under the Y loads' latency
                float* fbn = reinterpret_cast<float*>(Z + H * ZS);   // 16 B behind the plane (c2r_lds)
                const int wv = tid >> 6;
                if (wv < 2) {
                    float fs, fh;
                    ffc::bn_fold_channel(a.bn_fold, 2 * ch + wv, plane < a.C, fs, fh);
                    if ((tid & 63) == 0) {
                        fbn[2 * wv] = fs;
                        fbn[2 * wv + 1] = fh;
                        if (plane == 0 && wv == 0 && a.bn_fold.update_running) *a.bn_fold.num_batches_tracked += 1;
                    }
                }
                __syncthreads();
                bsr = fbn[0];
                bhr = fbn[1];
                bsi = fbn[2];
                bhi = fbn[3];
            }
            if constexpr (RPRE) {
                if (a.residual) {
                    const int jj = tid % N1;
#pragma unroll
                    for (int rd = 0; rd < RROUNDS; ++rd) {
                        const int g = rd * RLPR + tid / N1;
#pragma unroll
                        for (int i = 0; i < RITER; ++i) {
                            const int q4 = jj + N1 * i;
                            const int rr = q4 / (W / 4), x = 4 * (q4 % (W / 4));
                            const int y = 2 * g + rr;
                            const bool ok = g < H / 2 && q4 < 2 * W / 4;
                            res[rd][i] = *reinterpret_cast<const float2*>(tpl + (ok ? (y / 2) * tW + x / 2 : 0));
                        }
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < NL; ++u) {
                const int i = u * FU2_THREADS + tid;
                if (i < N4) {
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        float2 z = e ? make_float2(v[u].z, v[u].w) : make_float2(v[u].x, v[u].y);
                        const int f = 2 * i + e, r = f / WP, k = f - r * WP;
                        if (bn) z = make_float2(fmaxf(fmaf(z.x, bsr, bhr), 0.0f), fmaxf(fmaf(z.y, bsi, bhi), 0.0f));
                        Z[r * ZS + k] = z;
                    }
                }
            }
        } else {
            const float* pre = a.Y + (size_t)plane * 2 * H * WP;   // PLANAR: Re plane, Im plane behind it
            for (int i0 = 0; i0 < H * WP; i0 += 16 * FU2_THREADS) {
                float2 v[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    const int i = i0 + u * FU2_THREADS + tid;
                    if (i < H * WP) {
                        const int k = i % WP;
                        const float isc = (k == 0 || 2 * k == W) ? 1.0f : a.iscale;
                        v[u] = make_float2(pre[i] * isc, pre[H * WP + i] * isc);
                    }
                }
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    const int i = i0 + u * FU2_THREADS + tid;
                    if (i < H * WP) {
                        const int r = i / WP, k = i - r * WP;
                        if (bn) v[u] = make_float2(fmaxf(fmaf(v[u].x, bsr, bhr), 0.0f), fmaxf(fmaf(v[u].y, bsi, bhi), 0.0f));
                        Z[r * ZS + k] = v[u];
                    }
                }
            }
        }
    }
    __syncthreads();

    // 2. inverse columns (length H).  The row C2R keeps only Re of columns 0 and W/2 after this pass,
    //    and Re(IFFT(a)) = IFFT(a_h) with a_h[k] = (a[k] + conj(a[-k])) / 2 (real), so those two
    //    columns run as ONE complex IFFT of z = a_h + i b_h placed in the pad column WP: W/2 lines
    //    instead of W/2 + 1 (whole rounds of the column pass: 128^2 3 -> 2, 64^2 2 -> 1).
    static_assert(ZS > WP, "pad column for the packed DC / Nyquist column");
    for (int r = tid; r < H; r += FU2_THREADS) {
        const int rm = (H - r) & (H - 1);
        const float2 a0 = Z[r * ZS], a1 = Z[rm * ZS], b0 = Z[r * ZS + W / 2], b1 = Z[rm * ZS + W / 2];
        const float ahx = 0.5f * (a0.x + a1.x), ahy = 0.5f * (a0.y - a1.y);
        const float bhx = 0.5f * (b0.x + b1.x), bhy = 0.5f * (b0.y - b1.y);
        Z[r * ZS + WP] = make_float2(ahx - bhy, ahy + bhx);
    }
    __syncthreads();
#ifndef FFC_C2R_SKIP_COL   // timing probes only (tools/build_variant.sh): results are wrong without it
    {
        constexpr int N1c = Split<H>::N1, LPR = FU2_THREADS / N1c;
        const int jj = tid % N1c;
        for (int l0 = 0; l0 < W / 2; l0 += LPR) {
            const int l = l0 + tid / N1c;
            if (l < W / 2) line_fft<H, true>(Z + (l == 0 ? WP : l), ZS, jj, twc);
        }
    }
#endif
    __syncthreads();

    // 3. rows two at a time: z[k] = A_ext[k] + i B_ext[k] (Hermitian extension of each half
    //    spectrum, Im of bins 0 and W/2 dropped) -> inverse FFT -> Re = row 2g, Im = row 2g+1
    {
        constexpr int LPR = RLPR;
        const int jj = tid % N1;
#pragma unroll
        for (int rd = 0; rd < RROUNDS; ++rd) {
            const int g = rd * LPR + tid / N1;
            if (g < H / 2) {
                float2* ra = Z + 2 * g * ZS;
                float2* rb = ra + ZS;
                float re[N2], im[N2];
#pragma unroll
                for (int m = 0; m < N2; ++m) {
                    const int k = jj + N1 * m;
                    float2 A, B;
                    if (k == 0 || k == W / 2) {   // Re parts from the packed column (step 2)
                        const float2 za = ra[WP], zb = rb[WP];
                        A = make_float2(k == 0 ? za.x : za.y, 0.0f);
                        B = make_float2(k == 0 ? zb.x : zb.y, 0.0f);
                    } else if (k < W / 2) {
                        A = ra[k];
                        B = rb[k];
                    } else {
                        A = ra[W - k];
                        B = rb[W - k];
                        A.y = -A.y;
                        B.y = -B.y;
                    }
                    re[m] = A.x - B.y;
                    im[m] = A.y + B.x;
                }
#ifndef FFC_C2R_SKIP_ROW
                stage_a<W, true>(re, im, twr);
                float ore[Q][N1], oim[Q][N1];
                stage_b<W, true>(ra, 1, re, im, jj, ore, oim);
#else
                float ore[Q][N1], oim[Q][N1];
#pragma unroll
                for (int q = 0; q < Q; ++q)
#pragma unroll
                    for (int k1 = 0; k1 < N1; ++k1) { ore[q][k1] = re[q * N1 + k1]; oim[q][k1] = im[q * N1 + k1]; }
#endif
                float* fa = reinterpret_cast<float*>(ra);   // 4*ZS >= 2W floats: row 2g then row 2g+1
#pragma unroll
                for (int q = 0; q < Q; ++q)
#pragma unroll
                    for (int k1 = 0; k1 < N1; ++k1) {
                        const int x = (jj + N1 * q) + N2 * k1;
                        fa[x] = ore[q][k1];
                        fa[W + x] = oim[q][k1];
                    }
                wave_lds_sync();   // both output rows are in LDS before the lanes read them as float4
                // scale, residual, store (float4 per lane, the group covers both rows)
#pragma unroll
                for (int i = 0; i < (2 * W / 4 + N1 - 1) / N1; ++i) {
                    const int q4 = jj + N1 * i;
                    if (q4 < 2 * W / 4) {
                        const int rr = q4 / (W / 4);
                        const int x = 4 * (q4 % (W / 4));
                        const int y = 2 * g + rr;
                        float4 v = *reinterpret_cast<const float4*>(fa + rr * W + x);
                        v.x *= a.norm;
                        v.y *= a.norm;
                        v.z *= a.norm;
                        v.w *= a.norm;
                        if (a.residual) {
                            const float* trow = tpl + (y / UP) * tW;
                            if constexpr (UP == 1) {
                                const float4 s = *reinterpret_cast<const float4*>(trow + x);
                                v.x += in_tf(s.x, sc, sh, a.in_relu);
                                v.y += in_tf(s.y, sc, sh, a.in_relu);
                                v.z += in_tf(s.z, sc, sh, a.in_relu);
                                v.w += in_tf(s.w, sc, sh, a.in_relu);
                            } else {
                                float2 s;
                                if constexpr (RPRE) {
                                    s = res[rd][i];
                                } else {
                                    s = *reinterpret_cast<const float2*>(trow + x / 2);
                                }
                                const float s0 = in_tf(s.x, sc, sh, a.in_relu), s1 = in_tf(s.y, sc, sh, a.in_relu);
                                v.x += s0;
                                v.y += s0;
                                v.z += s1;
                                v.w += s1;
                            }
                        }
                        *reinterpret_cast<float4*>(opl + (size_t)y * W + x) = v;
                    }
                }
            }
        }
    }
}

// ---------------------------------------------------------------- stage 2: spectral mix
struct MixArgs {
    const float* T;
    const float* wmixT;   // (2C, Mpad) transposed, zero padded
    float* slab;          // pass 0: [B*nsplit][2C] float4
    const float* bn_scale;
    const float* bn_shift;
    float* Y;             // pass 1: (B, C, H, WP) float2
    int B, C, H, W, up, nsplit, ntiles, Mpad;
    float norm;
};

constexpr int MIX_TILES_PER_WG = 32;   // 8 per wave: amortises the weight staging

// Geometry of one sample's spectrum as the mix sees it (rebuilt from T, see the file comment).
struct MixGeom {
    const float2* Tb;   // this sample's T
    size_t planeT;      // complex bins per channel of T
    int WP, NB, h, w, WPt, up, tstepH, tstepW;
    float norm;
};

// source index in T, conjugation and factor f = X / T of flat bin n (zero factor beyond the plane)
__device__ __forceinline__ void bin_params(const MixGeom& g, int n, int& idx, bool& cj, float& fr, float& fi) {
    idx = 0;
    cj = false;
    fr = 0.0f;
    fi = 0.0f;
    if (n < g.NB) {
        const int kh = n / g.WP, kw = n - kh * g.WP;
        if (g.up == 1) {
            idx = n;
            fr = g.norm;
        } else {
            const int khp = kh & (g.h - 1), kwp = kw & (g.w - 1);
            if (kwp <= g.w / 2) {
                idx = khp * g.WPt + kwp;
            } else {
                idx = ((g.h - khp) & (g.h - 1)) * g.WPt + (g.w - kwp);
                cj = true;
            }
            const float c1 = 1.0f + c_twc[kh * g.tstepH], s1 = -c_tws[kh * g.tstepH];
            const float c2 = 1.0f + c_twc[kw * g.tstepW], s2 = -c_tws[kw * g.tstepW];
            fr = (c1 * c2 - s1 * s2) * g.norm;
            fi = (c1 * s2 + s1 * c2) * g.norm;
        }
    }
}

// F16 (config 5, "fp16 MFMA channel-mix"): the weights (fp16 [Mpad][2C]) and the rebuilt spectrum
// are rounded to fp16 and multiplied on v_mfma_f32_32x32x16_f16 with fp32 accumulation; lane (h, r)
// of k-block kb carries channels 8kb + 4h + 0..3 as (Re, Im) pairs.  Needs CC % 8 == 0.
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

// The wave's A operand: fp32 fragments in registers (compile-time C, C*MT <= 64), fp16 fragments in
// registers (F16), or read from the LDS copy Wm per k-step.
#ifdef FFC_MIX_F32   // A/B measurement builds: the register-resident fp32 mix on the f32-input MFMA
constexpr bool MIX_SPLIT = false;
#else
constexpr bool MIX_SPLIT = true;
#endif

template <int MT, int CC, bool F16, bool NOAREG = false, bool SPLITOK = true>
struct MixA {
    static constexpr bool AREG = !NOAREG && !F16 && CC > 0 && CC * MT <= 64;
    // fp32 mix with register-resident weights: fp32-accurate split-bf16 products (ffc_internal.h
    // split3), the weights split once per workgroup; element j of lane half hh in k-block q is
    // k = 2 (8q + j) + hh, i.e. channel 8q + j, Re (hh = 0) or Im (hh = 1)
    static constexpr bool SPLIT = AREG && MIX_SPLIT && SPLITOK && CC % 8 == 0;
    float areg[AREG ? CC : 1][MT];
    Split3 as3[SPLIT ? CC / 8 : 1][SPLIT ? MT : 1];
    half8 a16[F16 ? MT : 1][F16 ? CC / 8 : 1];
    const float* Wm;
    int Mpad;
    __device__ void load(const float* Wm_, const void* wsrc, int Mpad_, int C2, int hh, int col) {
        Wm = Wm_;
        Mpad = Mpad_;
        if constexpr (F16) {   // straight from L2: W16[o][k], 8 consecutive k
            const _Float16* W16 = reinterpret_cast<const _Float16*>(wsrc);
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int kb = 0; kb < CC / 8; ++kb)
                    a16[mt][kb] = *reinterpret_cast<const half8*>(W16 + (size_t)(mt * 32 + col) * C2 + 16 * kb + 8 * hh);
        }
        if constexpr (AREG) {
#pragma unroll
            for (int s = 0; s < CC; ++s)
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) areg[s][mt] = Wm[(2 * s + hh) * Mpad + mt * 32 + col];
        }
        if constexpr (SPLIT) {
#pragma unroll
            for (int q = 0; q < CC / 8; ++q)
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    float av[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) av[j] = areg[8 * q + j][mt];
                    as3[q][mt] = split3(av);
                }
        }
    }
};

// acc[mt] = Wmix[mt rows] . Z[:, bin n of this lane] (Z rebuilt from T on the fly)
template <int MT, int CC, bool F16, bool NOAREG = false, bool SPLITOK = true>
__device__ __forceinline__ void mix_tile(floatx16 (&acc)[MT], const MixGeom& g, const MixA<MT, CC, F16, NOAREG, SPLITOK>& A, int n,
                                         int C, int hh, int col) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[mt][r] = 0.0f;
    int idx;
    bool cj;
    float fr, fi;
    bin_params(g, n, idx, cj, fr, fi);
    if constexpr (F16) {
        float2 tv[CC / 2];   // this lane half's channels 8kb + 4hh + q
#pragma unroll
        for (int kb = 0; kb < CC / 8; ++kb)
#pragma unroll
            for (int q = 0; q < 4; ++q) tv[kb * 4 + q] = g.Tb[idx + (size_t)(8 * kb + 4 * hh + q) * g.planeT];
#pragma unroll
        for (int kb = 0; kb < CC / 8; ++kb) {
            half8 bz;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float2 t2 = tv[kb * 4 + q];
                if (cj) t2.y = -t2.y;
                bz[2 * q] = (_Float16)(t2.x * fr - t2.y * fi);
                bz[2 * q + 1] = (_Float16)(t2.x * fi + t2.y * fr);
            }
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
                acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A.a16[mt][kb], bz, acc[mt], 0, 0, 0);
        }
    } else if constexpr (MixA<MT, CC, F16, NOAREG, SPLITOK>::SPLIT) {
        float2 tv[CC];
#pragma unroll
        for (int s = 0; s < CC; ++s) tv[s] = g.Tb[idx + (size_t)s * g.planeT];
#pragma unroll
        for (int q = 0; q < CC / 8; ++q) {
            float zb[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float2 t2 = tv[8 * q + j];
                if (cj) t2.y = -t2.y;
                zb[j] = hh ? (t2.x * fi + t2.y * fr) : (t2.x * fr - t2.y * fi);
            }
            const Split3 bs = split3(zb);
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) acc[mt] = mfma_split3(A.as3[q][mt], bs, acc[mt]);
        }
    } else if constexpr (CC > 0) {
        // all C gathered loads of the tile issued before its MFMAs (a register prefetch of the next
        // tile measured slower: 276 VGPRs, one wave per SIMD)
        float2 tv[CC];
#pragma unroll
        for (int s = 0; s < CC; ++s) tv[s] = g.Tb[idx + (size_t)s * g.planeT];
#pragma unroll
        for (int s = 0; s < CC; ++s) {
            float2 t2 = tv[s];
            if (cj) t2.y = -t2.y;
            const float z = hh ? (t2.x * fi + t2.y * fr) : (t2.x * fr - t2.y * fi);
            if constexpr (MixA<MT, CC, F16, NOAREG, SPLITOK>::AREG) {
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
                    acc[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(A.areg[s][mt], z, acc[mt], 0, 0, 0);
            } else {
                const float* wr = A.Wm + (2 * s + hh) * A.Mpad + col;
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
                    acc[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(wr[mt * 32], z, acc[mt], 0, 0, 0);
            }
        }
    } else {
        const float2* tp = g.Tb + idx;
        for (int s0 = 0; s0 < C; s0 += 8) {
            float z[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                float2 tv = make_float2(0.0f, 0.0f);
                if (s0 + u < C) tv = tp[(size_t)(s0 + u) * g.planeT];
                if (cj) tv.y = -tv.y;
                const float xr = tv.x * fr - tv.y * fi;
                const float xi = tv.x * fi + tv.y * fr;
                z[u] = hh ? xi : xr;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int s = s0 + u;
                if (s < C) {
                    const float* wr = A.Wm + (2 * s + hh) * A.Mpad + col;
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt)
                        acc[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(wr[mt * 32], z[u], acc[mt], 0, 0, 0);
                }
            }
        }
    }
}

__device__ __forceinline__ MixGeom mix_geom(const MixArgs& a, int b, int C) {
    MixGeom g;
    const int H = a.H, W = a.W;
    g.WP = W / 2 + 1;
    g.NB = H * g.WP;
    g.h = H / a.up;
    g.w = W / a.up;
    g.WPt = g.w / 2 + 1;
    g.planeT = (size_t)g.h * g.WPt;
    g.Tb = reinterpret_cast<const float2*>(a.T) + (size_t)b * C * g.planeT;
    g.up = a.up;
    g.tstepH = 128 / H;
    g.tstepW = 128 / W;
    g.norm = a.norm;
    return g;
}

// CC: compile-time channel count (0: runtime a.C) -- with it the k-loop unrolls fully and all C
// gathered B loads of a tile are issued before its MFMAs
template <int MT, int PASS, int CC = 0, bool F16 = false>
__global__ __launch_bounds__(FU2_THREADS) void fu2d_mix_kernel(MixArgs a) {
    static_assert(!F16 || (CC > 0 && CC % 8 == 0), "fp16 mix: compile-time C, multiple of 8");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int C = CC ? CC : a.C, C2 = 2 * C;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int hh = lane >> 5, col = lane & 31;
    // sample-major within an XCD: consecutive ids go to consecutive XCDs, so b = id % B keeps a
    // sample's workgroups (and its T) on one XCD's L2 when B % 8 == 0
    const int b = blockIdx.x % a.B;
    const int split = blockIdx.x / a.B;
    const int t_lo = (int)((long long)split * a.ntiles / a.nsplit);
    const int t_hi = (int)((long long)(split + 1) * a.ntiles / a.nsplit);

    float* Wm = smem;                                         // (2C, Mpad), whole 64-lane DMA groups
    float* bnss = F16 ? smem : smem + (C2 * a.Mpad + 255) / 256 * 256;   // pass 1: scale [2C] | shift [2C]
    float* scr = bnss;                                        // pass 0: per-wave tile scratch + merge area
    if constexpr (!F16) ffc::dma_copy16(a.wmixT, Wm, (C2 * a.Mpad) >> 2, tid, FU2_THREADS);
    if constexpr (PASS == 1) {
        for (int i = tid; i < C2; i += FU2_THREADS) {
            bnss[i] = a.bn_scale[i];
            bnss[C2 + i] = a.bn_shift[i];
        }
    }
    ffc::dma_wait();
    __syncthreads();
    MixA<MT, CC, F16> A;
    A.load(Wm, a.wmixT, a.Mpad, C2, hh, col);
    const MixGeom g = mix_geom(a, b, C);
    const int NB = g.NB;

    float st_n[MT], st_mean[MT], st_m2[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) st_n[mt] = st_mean[mt] = st_m2[mt] = 0.0f;

    for (int tile = t_lo + wave; tile < t_hi; tile += FU2_THREADS / 64) {
        const int n = tile * 32 + col;
        const bool valid = n < NB;
        floatx16 acc[MT];
        mix_tile<MT, CC, F16>(acc, g, A, n, C, hh, col);
        if constexpr (PASS == 0) {
            if (a.Y) {   // spill: the raw mix output, BN + ReLU applied by the C2R that reads it
                float2* Yb = reinterpret_cast<float2*>(a.Y) + (size_t)b * C * NB;
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int r = 0; r < 16; r += 2) {
                        const int o = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;   // even: Re, o+1: Im
                        if (valid && o < C2) Yb[(size_t)(o >> 1) * NB + n] = make_float2(acc[mt][r], acc[mt][r + 1]);
                    }
            }
            const int nv = min(32, NB - tile * 32);
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                float mean, m2;
                ffc::tile_row_stats(acc[mt], nv, scr + wave * ffc::TILE_SCRATCH, mean, m2);
                const float cn = (float)nv;
                const float tot = st_n[mt] + cn;
                const float delta = mean - st_mean[mt];
                st_mean[mt] += delta * (cn / tot);
                st_m2[mt] += m2 + delta * delta * (st_n[mt] * cn / tot);
                st_n[mt] = tot;
            }
        } else {
            float2* Yb = reinterpret_cast<float2*>(a.Y) + (size_t)b * C * NB;
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int r = 0; r < 16; r += 2) {
                    const int o = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;   // even: Re, o+1: Im
                    if (valid && o < C2) {
                        const float re = fmaxf(fmaf(acc[mt][r], bnss[o], bnss[C2 + o]), 0.0f);
                        const float im = fmaxf(fmaf(acc[mt][r + 1], bnss[o + 1], bnss[C2 + o + 1]), 0.0f);
                        Yb[(size_t)(o >> 1) * NB + n] = make_float2(re, im);
                    }
                }
        }
    }

    if constexpr (PASS == 0) {
        // merge the 4 waves' partials (fixed order) -> slab row blockIdx.x
        __syncthreads();
        float4* mg = reinterpret_cast<float4*>(scr);   // [wave][MT*32]
        if ((lane & 1) == 0) {
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
                mg[wave * MT * 32 + mt * 32 + (lane >> 1)] = make_float4(st_n[mt], st_mean[mt], st_m2[mt], 0.0f);
        }
        __syncthreads();
        for (int o = tid; o < C2; o += FU2_THREADS) {
            float nn = 0.0f, mean = 0.0f, m2 = 0.0f;
            for (int wv = 0; wv < FU2_THREADS / 64; ++wv) {
                const float4 e = mg[wv * MT * 32 + o];
                if (e.x > 0.0f) {
                    const float tot = nn + e.x;
                    const float delta = e.y - mean;
                    mean += delta * (e.x / tot);
                    m2 += e.z + delta * delta * (nn * e.x / tot);
                    nn = tot;
                }
            }
            reinterpret_cast<float4*>(a.slab)[(size_t)blockIdx.x * C2 + o] = make_float4(nn, mean, m2, 0.0f);
        }
    }
}

// ---------------------------------------------------------------- r2c + mix pass 0 in one launch
// Small t planes (HT = 8 or 16, the gen64 generator's ffc2 / ffc3 Fourier units at the per-rank
// batches of strong scaling): every mix workgroup recomputes its sample's T -- bn1 (+ ReLU) of the
// C planes, row FFTs (one row per thread), column FFTs (one column line per thread), all in LDS --
// instead of reading it from a separate r2c launch.  The sample is 8-16 KB and its FFTs are a few
// hundred VALU per thread, so the repeat per bin-range workgroup costs less than a kernel boundary
// plus the r2c's own latency chain (B x C workgroups of one small plane each).  bn1 is finalized
// here from its whole slab (ffc::bn_fold_block; workgroup 0 leads); T stays in LDS.  Then exactly
// mix pass 0 with the spilled raw Y (the C2R applies the FU's BN on load).
struct R2cMixArgs {
    MixArgs m;
    const float* t;          // (B, C, HT, HT)
    const float* in_scale;   // bn1 affine (or has_fold)
    const float* in_shift;
    int in_relu, has_fold;
    ffc_bn_fold fold;
};

template <int HT, int CC>
struct R2cMixLds {
    static constexpr int WPt = HT / 2 + 1, PT = HT * WPt;
    static constexpr int MPAD = (2 * CC + 31) / 32 * 32;
    static constexpr int WM = (2 * CC * MPAD + 255) / 256 * 256;       // mix weight (DMA groups)
    static constexpr int SCR = (FU2_THREADS / 64) * ffc::TILE_SCRATCH;  // tile stats / merge
    static constexpr int TL = 2 * CC * PT;                             // T (float2)
    static constexpr int R = CC * HT * HT;                             // transformed real planes
    static constexpr int FLOATS = WM + SCR + TL + R + 2 * CC;
};

#ifdef FFC_R2CMIX_DUMP   // DESIGN 10c probe build: Tl after the row FFTs (slot 0) and at the end (slot 1)
__device__ float g_r2cmix_dump[512 * 2 * 4608];
#endif
#if defined(FFC_R2CMIX_CANARY) || defined(FFC_R2CMIX_FCANARY)
__device__ int g_r2cmix_canary_hits;
#endif
#if defined(FFC_R2CMIX_DBG) || defined(FFC_R2CMIX_DBGEND)
// DESIGN 10c probe build: per workgroup, per channel: bn1 scale, shift, sum R, sum |T| after the row
// FFTs, sum |T| after the column FFTs (thread ch sums its channel in a fixed order)
__device__ float g_r2cmix_dbg[4096 * 5 * 32];
#define R2CMIX_DBG(slot, expr_of_ch)                                                        \
    do {                                                                                    \
        __syncthreads();                                                                    \
        if (tid < C) {                                                                      \
            const int ch = tid;                                                             \
            g_r2cmix_dbg[((size_t)blockIdx.x * 5 + (slot)) * 32 + ch] = (expr_of_ch);       \
        }                                                                                   \
        __syncthreads();                                                                    \
    } while (0)
template <int N>
__device__ float dbg_sum(const float* p, int stride) {
    float s = 0.0f;
    for (int i = 0; i < N; ++i) s += fabsf(p[i * stride]);
    return s;
}
#endif
#ifndef FFC_R2CMIX_DBG
#undef R2CMIX_DBG
#define R2CMIX_DBG(slot, e) do { } while (0)
#endif

template <int MT, int CC, int HT>
__global__ __launch_bounds__(FU2_THREADS) void fu2d_r2c_mix_kernel(R2cMixArgs ra) {
    using LY = R2cMixLds<HT, CC>;
    constexpr int C = CC, C2 = 2 * CC, WPt = LY::WPt, PT = LY::PT;
    static_assert((CC & (CC - 1)) == 0 && CC <= FU2_THREADS / 4 && (C * HT * HT) % (4 * FU2_THREADS) == 0,
                  "whole float4 rounds of the sample");
    const MixArgs& a = ra.m;
#ifdef FFC_R2CMIX_FRONTPAD   // DESIGN 10c probe: unused LDS IN FRONT of the layout
    extern __shared__ __attribute__((aligned(16))) float smem_front[];
    float* const smem = smem_front + FFC_R2CMIX_FRONTPAD / 4;
#else
    extern __shared__ __attribute__((aligned(16))) float smem[];
#endif
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int hh = lane >> 5, col = lane & 31;
    const int b = blockIdx.x % a.B;
    const int split = blockIdx.x / a.B;
    const int t_lo = (int)((long long)split * a.ntiles / a.nsplit);
    const int t_hi = (int)((long long)(split + 1) * a.ntiles / a.nsplit);
    float* Wm = smem;
    float* scr = smem + LY::WM;
    float2* Tl = reinterpret_cast<float2*>(scr + LY::SCR);
    float* R = scr + LY::SCR + LY::TL;
    float* fss = R + LY::R;   // bn1 scale [C] | shift [C]

    // 1. the sample's t planes (registers) and the mix weight (LDS-DMA), all in flight
    constexpr int NV = C * HT * HT / 4 / FU2_THREADS;
    const float4* src = reinterpret_cast<const float4*>(ra.t + (size_t)b * C * HT * HT);
#if defined(FFC_R2CMIX_ZERO_LDS) || defined(FFC_R2CMIX_ZERO_SCR)   // DESIGN 10c probes
#ifdef FFC_R2CMIX_ZERO_LDS
    for (int i = tid; i < LY::FLOATS; i += FU2_THREADS) smem[i] = 0.0f;
#else
    for (int i = tid; i < LY::SCR; i += FU2_THREADS) scr[i] = 0.0f;
#endif
    __syncthreads();
#endif
#ifdef FFC_R2CMIX_CANARY   // DESIGN 10c probe: a canary in the LDS padding behind the layout (FFC_R2CMIX_PAD)
    for (int i = tid; i < FFC_R2CMIX_PAD / 4; i += FU2_THREADS) smem[LY::FLOATS + i] = __int_as_float(0x7fc0dead);
    __syncthreads();
#endif
#ifdef FFC_R2CMIX_FCANARY  // DESIGN 10c probe: a canary in the LDS padding in front of the layout (FFC_R2CMIX_FRONTPAD)
    for (int i = tid; i < FFC_R2CMIX_FRONTPAD / 4; i += FU2_THREADS) smem_front[i] = __int_as_float(0x7fc0beef);
    __syncthreads();
#endif
#ifdef FFC_R2CMIX_V192    // DESIGN 10c probe: 192 VGPRs reserved -> at most two workgroups per CU, layout unpadded
    asm volatile("" ::: "v191");
#endif
    float4 v[NV];
#ifndef FFC_R2CMIX_LATE_T
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] = src[j * FU2_THREADS + tid];
#endif
#ifdef FFC_R2CMIX_NODMA   // DESIGN 10c probe: the mix weight through registers instead of LDS-DMA
    for (int i = tid; i < (C2 * a.Mpad) >> 2; i += FU2_THREADS)
        reinterpret_cast<float4*>(Wm)[i] = reinterpret_cast<const float4*>(a.wmixT)[i];
#else
    ffc::dma_copy16(a.wmixT, Wm, (C2 * a.Mpad) >> 2, tid, FU2_THREADS);
#endif
    // 2. bn1 (under the loads' latency): the whole-slab fold, scratch in the (not yet used) tile-stats
    //    area.  The per-channel fold (ffc::bn_fold_channels, as in the staged r2c) was measured
    //    non-deterministic here -- T of two channels wrong in a few workgroups per launch (r05i,
    //    tools/experiments/r2cmix_*.py) -- and bn_fold_block is not.
    if (ra.has_fold) {
#ifdef FFC_R2CMIX_CHFOLD
#ifdef FFC_R2CMIX_DMA_WAIT
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
#ifdef FFC_R2CMIX_PREBAR
        __syncthreads();
#endif
#ifdef FFC_R2CMIX_WAVE0   // DESIGN 10c probe: wave 0 alone folds (64 / C lanes per channel)
        constexpr int L = 64 / C;
        if (tid < 64) {
#else
        constexpr int L = FU2_THREADS / C;
        {
#endif
        float s_, h_;
        const int o = tid / L;
#ifdef FFC_R2CMIX_NOLEAD
        constexpr bool lead = false;
#else
        const bool lead = blockIdx.x == 0;
#endif
        ffc::bn_fold_channels<L>(ra.fold, o, lead, s_, h_);
        if ((tid & (L - 1)) == 0) {
            fss[o] = s_;
            fss[C + o] = h_;
        }
        if (lead && tid == 0 && ra.fold.update_running) *ra.fold.num_batches_tracked += 1;
        }
#ifdef FFC_R2CMIX_NOP
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#endif
#else
        ffc::bn_fold_block<FU2_THREADS>(ra.fold, fss, fss + C, blockIdx.x == 0, reinterpret_cast<double*>(scr));
#endif
    } else if (tid < C) {
        fss[tid] = ra.in_scale ? ra.in_scale[tid] : 1.0f;
        fss[C + tid] = ra.in_scale ? ra.in_shift[tid] : 0.0f;
    }
    ffc::dma_wait();
    __syncthreads();
#ifdef FFC_R2CMIX_LATE_T
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] = src[j * FU2_THREADS + tid];
#endif
    // 3. s0 = relu(t * scale + shift) -> R
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int i = j * FU2_THREADS + tid;
        const int ch = (4 * i) / (HT * HT);
        const float sc = fss[ch], sh = fss[C + ch];
        float4 q = v[j];
        q.x = in_tf(q.x, sc, sh, ra.in_relu);
        q.y = in_tf(q.y, sc, sh, ra.in_relu);
        q.z = in_tf(q.z, sc, sh, ra.in_relu);
        q.w = in_tf(q.w, sc, sh, ra.in_relu);
        reinterpret_cast<float4*>(R)[i] = q;
    }
    __syncthreads();
    R2CMIX_DBG(0, fss[ch]);
    R2CMIX_DBG(1, fss[C + ch]);
    R2CMIX_DBG(2, (dbg_sum<HT * HT>(R + ch * HT * HT, 1)));
#if FFC_R2CMIX_XB == 3   // DESIGN 10c probes: one extra barrier after step 3 / 4 / 5
    __syncthreads();
#endif
    // 4. row FFTs (row r = channel * HT + y), bins 0..HT/2 -> Tl[r * WPt + k]
    for (int r = tid; r < C * HT; r += FU2_THREADS) {
        float re[HT], im[HT];
#pragma unroll
        for (int x4 = 0; x4 < HT / 4; ++x4) {
            const float4 q = reinterpret_cast<const float4*>(R + r * HT)[x4];
            re[4 * x4] = q.x;
            re[4 * x4 + 1] = q.y;
            re[4 * x4 + 2] = q.z;
            re[4 * x4 + 3] = q.w;
        }
#pragma unroll
        for (int x = 0; x < HT; ++x) im[x] = 0.0f;
        fft_reg<HT, false>(re, im);
#pragma unroll
        for (int k = 0; k < WPt; ++k) Tl[r * WPt + k] = make_float2(re[k], im[k]);
    }
    __syncthreads();
    R2CMIX_DBG(3, (dbg_sum<2 * PT>(reinterpret_cast<const float*>(Tl + ch * PT), 1)));
#ifdef FFC_R2CMIX_DUMP
    if (blockIdx.x < 512 && LY::TL <= 4608)
        for (int i = tid; i < LY::TL; i += FU2_THREADS)
            g_r2cmix_dump[((size_t)blockIdx.x * 2) * 4608 + i] = reinterpret_cast<const float*>(Tl)[i];
    __syncthreads();   // every wave's dump reads precede the column pass's writes
#endif
#if FFC_R2CMIX_XB == 4
    __syncthreads();
#endif
    // 5. column FFTs (line l = channel * WPt + k)
    for (int l = tid; l < C * WPt; l += FU2_THREADS) {
        const int ch = l / WPt, k = l - ch * WPt;
        float2* cp = Tl + ch * PT + k;
        float re[HT], im[HT];
#pragma unroll
        for (int y = 0; y < HT; ++y) {
            const float2 z = cp[y * WPt];
            re[y] = z.x;
            im[y] = z.y;
        }
        fft_reg<HT, false>(re, im);
#pragma unroll
        for (int y = 0; y < HT; ++y) cp[y * WPt] = make_float2(re[y], im[y]);
    }
    __syncthreads();
    R2CMIX_DBG(4, (dbg_sum<2 * PT>(reinterpret_cast<const float*>(Tl + ch * PT), 1)));
#if FFC_R2CMIX_XB == 5
    __syncthreads();
#endif

    // 6. mix pass 0 on T in LDS: raw Y spill + BN partials (as fu2d_mix_kernel<MT, 0, CC>)
    MixA<MT, CC, false> A;
    A.load(Wm, a.wmixT, a.Mpad, C2, hh, col);
    MixGeom g = mix_geom(a, b, C);
    g.Tb = Tl;
    const int NB = g.NB;
    float st_n[MT], st_mean[MT], st_m2[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) st_n[mt] = st_mean[mt] = st_m2[mt] = 0.0f;
    for (int tile = t_lo + wave; tile < t_hi; tile += FU2_THREADS / 64) {
        const int n = tile * 32 + col;
        const bool valid = n < NB;
        floatx16 acc[MT];
        mix_tile<MT, CC, false>(acc, g, A, n, C, hh, col);
        float2* Yb = reinterpret_cast<float2*>(a.Y) + (size_t)b * C * NB;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
                const int o = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;   // even: Re, o+1: Im
                if (valid && o < C2) Yb[(size_t)(o >> 1) * NB + n] = make_float2(acc[mt][r], acc[mt][r + 1]);
            }
        const int nv = min(32, NB - tile * 32);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            float mean, m2;
            ffc::tile_row_stats(acc[mt], nv, scr + wave * ffc::TILE_SCRATCH, mean, m2);
            const float cn = (float)nv;
            const float tot = st_n[mt] + cn;
            const float delta = mean - st_mean[mt];
            st_mean[mt] += delta * (cn / tot);
            st_m2[mt] += m2 + delta * delta * (st_n[mt] * cn / tot);
            st_n[mt] = tot;
        }
    }
    __syncthreads();
    float4* mg = reinterpret_cast<float4*>(scr);   // [wave][MT*32]
    if ((lane & 1) == 0) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
            mg[wave * MT * 32 + mt * 32 + (lane >> 1)] = make_float4(st_n[mt], st_mean[mt], st_m2[mt], 0.0f);
    }
    __syncthreads();
    for (int o = tid; o < C2; o += FU2_THREADS) {
        float nn = 0.0f, mean = 0.0f, m2 = 0.0f;
        for (int wv = 0; wv < FU2_THREADS / 64; ++wv) {
            const float4 e = mg[wv * MT * 32 + o];
            if (e.x > 0.0f) {
                const float tot = nn + e.x;
                const float delta = e.y - mean;
                mean += delta * (e.x / tot);
                m2 += e.z + delta * delta * (nn * e.x / tot);
                nn = tot;
            }
        }
        reinterpret_cast<float4*>(a.slab)[(size_t)blockIdx.x * C2 + o] = make_float4(nn, mean, m2, 0.0f);
#ifdef FFC_R2CMIX_DBGEND   // DESIGN 10c probe: the workgroup's stage checksums, taken at its very end
        g_r2cmix_dbg[((size_t)blockIdx.x * 5 + 3) * 32 + o] = m2;
#endif
    }
#ifdef FFC_R2CMIX_DUMP
    __syncthreads();
    if (blockIdx.x < 512 && LY::TL <= 4608)
        for (int i = tid; i < LY::TL; i += FU2_THREADS)
            g_r2cmix_dump[((size_t)blockIdx.x * 2 + 1) * 4608 + i] = reinterpret_cast<const float*>(Tl)[i];
#endif
#ifdef FFC_R2CMIX_CANARY
    __syncthreads();
    {
        int first = -1, cnt = 0;
        for (int i = tid; i < FFC_R2CMIX_PAD / 4; i += FU2_THREADS)
            if (__float_as_int(smem[LY::FLOATS + i]) != 0x7fc0dead) {
                if (first < 0) first = i;
                ++cnt;
            }
        if (cnt && atomicAdd(&g_r2cmix_canary_hits, 1) < 40)
            printf("r2cmix canary: blk %d tid %d first pad float %d (layout float %d) count %d\n", (int)blockIdx.x,
                   tid, first, LY::FLOATS + first, cnt);
    }
#endif
#ifdef FFC_R2CMIX_FCANARY
    __syncthreads();
    {
        int last = -1, cnt = 0;
        for (int i = tid; i < FFC_R2CMIX_FRONTPAD / 4; i += FU2_THREADS)
            if (__float_as_int(smem_front[i]) != 0x7fc0beef) {
                last = i;
                ++cnt;
            }
        if (cnt && atomicAdd(&g_r2cmix_canary_hits, 1) < 40)
            printf("r2cmix front canary: blk %d tid %d last pad float %d (layout offset %d) count %d\n",
                   (int)blockIdx.x, tid, last, last - FFC_R2CMIX_FRONTPAD / 4, cnt);
    }
#endif
#ifdef FFC_R2CMIX_DBGEND
    __syncthreads();
    if (tid < C) {
        const int ch = tid;
        g_r2cmix_dbg[((size_t)blockIdx.x * 5 + 0) * 32 + ch] = fss[ch];
        g_r2cmix_dbg[((size_t)blockIdx.x * 5 + 1) * 32 + ch] = fss[C + ch];
        g_r2cmix_dbg[((size_t)blockIdx.x * 5 + 2) * 32 + ch] = dbg_sum<HT * HT>(R + ch * HT * HT, 1);
        g_r2cmix_dbg[((size_t)blockIdx.x * 5 + 4) * 32 + ch] =
            dbg_sum<2 * PT>(reinterpret_cast<const float*>(Tl + ch * PT), 1);
    }
#endif
}

// ---------------------------------------------------------------- pass 1 + inverse column FFT
// Mix pass 1 for HC = H in {32, 64, 128} with the C2R's inverse column FFT fused in: a workgroup
// owns whole spectral columns (CPW = 128 / HC columns, TPC = HC / 32 bin tiles each, one tile per
// wave), so after BN + ReLU the columns are in LDS and the length-HC inverse FFTs run there -- VALU /
// LDS work beside the MFMA-bound mix -- and the column-transformed spectrum goes out column-major
// Yc (B, C, W/2+1, H).  The C2R that follows is then rows only (fu2d_c2r_rows_kernel).
template <int MT, int CC, bool F16, int HC>
__global__ __launch_bounds__(FU2_THREADS) void fu2d_mix_cols_kernel(MixArgs a) {
    static_assert(CC > 0 && HC >= 32 && HC <= 128, "column-fused mix: compile-time C, H in [32, 128]");
    constexpr int TPC = HC / 32, CPW = 4 / TPC, LS = HC + 4;   // LS: padded column stride (float2)
    constexpr int C = CC, C2 = 2 * CC;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int hh = lane >> 5, col = lane & 31;
    const int b = blockIdx.x % a.B, cg0 = blockIdx.x / a.B, gstride = a.nsplit;   // nsplit: workgroups per sample
    const int wfl = F16 ? 0 : (C2 * a.Mpad + 255) / 256 * 256;
    float* Wm = smem;
    float* bnss = smem + wfl;                                         // scale [2C] | shift [2C]
    float2* Ycol = reinterpret_cast<float2*>(smem + wfl + 4 * C);     // [C][CPW][LS]
    if constexpr (!F16) ffc::dma_copy16(a.wmixT, Wm, (C2 * a.Mpad) >> 2, tid, FU2_THREADS);
    for (int i = tid; i < C2; i += FU2_THREADS) {
        bnss[i] = a.bn_scale[i];
        bnss[C2 + i] = a.bn_shift[i];
    }
    ffc::dma_wait();
    __syncthreads();
    MixA<MT, CC, F16, false, false> A;   // f32-input MFMA here: the split measured slower (fewer waves)
    A.load(Wm, a.wmixT, a.Mpad, C2, hh, col);
    const MixGeom g = mix_geom(a, b, C);
    const int cs = wave / TPC, kb = wave % TPC;
    const int ncg = (g.WP + CPW - 1) / CPW;
    constexpr int N1 = Split<HC>::N1;
    const int jj = tid % N1;
    float2* Yc = reinterpret_cast<float2*>(a.Y);
    // column groups cg0, cg0 + gstride, ...: the weight staging above is paid once per workgroup
    for (int cg = cg0; cg < ncg; cg += gstride) {
        const int kw = cg * CPW + cs, kh = kb * 32 + col;
        const bool kwv = kw < g.WP;
        floatx16 acc[MT];
        mix_tile<MT, CC, F16, false, false>(acc, g, A, kwv ? kh * g.WP + kw : g.NB, C, hh, col);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
                const int o = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;   // even: Re, o+1: Im
                if (o < C2) {
                    const float re = fmaxf(fmaf(acc[mt][r], bnss[o], bnss[C2 + o]), 0.0f);
                    const float im = fmaxf(fmaf(acc[mt][r + 1], bnss[o + 1], bnss[C2 + o + 1]), 0.0f);
                    Ycol[((o >> 1) * CPW + cs) * LS + kh] = make_float2(re, im);
                }
            }
        __syncthreads();
        const LaneTw<HC> tw(jj);
        for (int l0 = 0; l0 < C * CPW; l0 += FU2_THREADS / N1) {   // inverse column FFTs (length HC)
            const int line = l0 + tid / N1;
            if (line < C * CPW) line_fft<HC, true>(Ycol + line * LS, 1, jj, tw);
        }
        __syncthreads();
        for (int i = tid; i < C * CPW * (HC / 2); i += FU2_THREADS) {
            const int line = i / (HC / 2), q = i - line * (HC / 2);
            const int ch = line / CPW, c2 = line - ch * CPW;
            const int kwo = cg * CPW + c2;
            if (kwo < g.WP) {
                const float2 v0 = Ycol[line * LS + 2 * q], v1 = Ycol[line * LS + 2 * q + 1];
                *reinterpret_cast<float4*>(Yc + (((size_t)b * C + ch) * g.WP + kwo) * HC + 2 * q) =
                    make_float4(v0.x, v0.y, v1.x, v1.y);
            }
        }
        __syncthreads();   // Ycol is rewritten by the next column group
    }
}

// Row C2R + residual from the column-transformed Yc (B, C, W/2+1, H): a workgroup takes RB rows of one
// plane (small LDS, many workgroups per CU to cover HBM latency); rows in pairs as in fu2d_c2r_kernel.
template <int H, int W, int UP>
__global__ __launch_bounds__(FU2_THREADS) void fu2d_c2r_rows_kernel(C2rArgs a) {
    constexpr int WP = W / 2 + 1;
    constexpr int ZS = zstride(WP);
    constexpr int RB = H < 64 ? H : 64;
    constexpr int N1 = Split<W>::N1, N2 = Split<W>::N2, Q = Split<W>::Q;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float2* Z = reinterpret_cast<float2*>(smem);
    const int plane = blockIdx.x / (H / RB), rb = blockIdx.x - plane * (H / RB);
    const int kh0 = rb * RB;
    const int ch = plane % a.C;
    const int tid = threadIdx.x;
    {   // Yc[plane][kw][kh0 .. kh0+RB) -> Z rows (16 loads in flight per thread per batch)
        const float2* src = reinterpret_cast<const float2*>(a.Y) + (size_t)plane * WP * H + kh0;
        for (int i0 = 0; i0 < WP * RB; i0 += 16 * FU2_THREADS) {
            float2 v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int i = i0 + u * FU2_THREADS + tid;
                if (i < WP * RB) {
                    const int kw = i / RB, r = i - kw * RB;
                    v[u] = src[(size_t)kw * H + r];
                }
            }
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int i = i0 + u * FU2_THREADS + tid;
                if (i < WP * RB) {
                    const int kw = i / RB, r = i - kw * RB;
                    Z[r * ZS + kw] = v[u];
                }
            }
        }
    }
    __syncthreads();
    const float sc = a.in_scale ? a.in_scale[ch] : 1.0f;
    const float sh = a.in_scale ? a.in_shift[ch] : 0.0f;
    constexpr int tW = W / UP;
    const float* tpl = a.t + (size_t)plane * (H / UP) * tW;
    float* opl = a.out + (size_t)plane * H * W;
    constexpr int LPR = FU2_THREADS / N1;
    const int jj = tid % N1;
    for (int g0 = 0; g0 < RB / 2; g0 += LPR) {
        const int g = g0 + tid / N1;
        if (g >= RB / 2) continue;
        float2* ra = Z + 2 * g * ZS;
        float2* rbp = ra + ZS;
        float re[N2], im[N2];
#pragma unroll
        for (int m = 0; m < N2; ++m) {
            const int k = jj + N1 * m;
            float2 Av, Bv;
            if (k <= W / 2) {
                Av = ra[k];
                Bv = rbp[k];
                if (k == 0 || k == W / 2) {
                    Av.y = 0.0f;
                    Bv.y = 0.0f;
                }
            } else {
                Av = ra[W - k];
                Bv = rbp[W - k];
                Av.y = -Av.y;
                Bv.y = -Bv.y;
            }
            re[m] = Av.x - Bv.y;
            im[m] = Av.y + Bv.x;
        }
        stage_a<W, true>(re, im, jj);
        float ore[Q][N1], oim[Q][N1];
        stage_b<W, true>(ra, 1, re, im, jj, ore, oim);
        float* fa = reinterpret_cast<float*>(ra);   // 4*ZS >= 2W floats: row 2g then row 2g+1
#pragma unroll
        for (int q = 0; q < Q; ++q)
#pragma unroll
            for (int k1 = 0; k1 < N1; ++k1) {
                const int x = (jj + N1 * q) + N2 * k1;
                fa[x] = ore[q][k1];
                fa[W + x] = oim[q][k1];
            }
        wave_lds_sync();   // both output rows are in LDS before the lanes read them as float4
#pragma unroll
        for (int i = 0; i < (2 * W / 4 + N1 - 1) / N1; ++i) {
            const int q4 = jj + N1 * i;
            if (q4 < 2 * W / 4) {
                const int rr = q4 / (W / 4);
                const int x = 4 * (q4 % (W / 4));
                const int y = kh0 + 2 * g + rr;
                float4 v = *reinterpret_cast<const float4*>(fa + rr * W + x);
                v.x *= a.norm;
                v.y *= a.norm;
                v.z *= a.norm;
                v.w *= a.norm;
                if (a.residual) {
                    const float* trow = tpl + (y / UP) * tW;
                    if constexpr (UP == 1) {
                        const float4 s4 = *reinterpret_cast<const float4*>(trow + x);
                        v.x += in_tf(s4.x, sc, sh, a.in_relu);
                        v.y += in_tf(s4.y, sc, sh, a.in_relu);
                        v.z += in_tf(s4.z, sc, sh, a.in_relu);
                        v.w += in_tf(s4.w, sc, sh, a.in_relu);
                    } else {
                        const float2 s2 = *reinterpret_cast<const float2*>(trow + x / 2);
                        const float s0 = in_tf(s2.x, sc, sh, a.in_relu), s1 = in_tf(s2.y, sc, sh, a.in_relu);
                        v.x += s0;
                        v.y += s0;
                        v.z += s1;
                        v.w += s1;
                    }
                }
                *reinterpret_cast<float4*>(opl + (size_t)y * W + x) = v;
            }
        }
    }
}

// ---------------------------------------------------------------- host side
bool pow2_in(int v, int lo, int hi) { return v >= lo && v <= hi && (v & (v - 1)) == 0; }

typedef void (*R2cKernel)(R2cArgs);
typedef void (*C2rKernel)(C2rArgs);
typedef void (*MixKernel)(MixArgs);

R2cKernel pick_r2c(int h, int w) {
    if (h != w) return nullptr;
    switch (h) {
        case 8: return fu2d_r2c_kernel<8, 8>;
        case 16: return fu2d_r2c_kernel<16, 16>;
        case 32: return fu2d_r2c_kernel<32, 32>;
        case 64: return fu2d_r2c_kernel<64, 64>;
        case 128: return fu2d_r2c_kernel<128, 128>;
    }
    return nullptr;
}

template <int N>
C2rKernel pick_c2r_up(int up) { return up == 1 ? fu2d_c2r_kernel<N, N, 1> : fu2d_c2r_kernel<N, N, 2>; }

C2rKernel pick_c2r(int H, int W, int up) {
    if (H != W) return nullptr;
    switch (H) {
        case 16: return pick_c2r_up<16>(up);
        case 32: return pick_c2r_up<32>(up);
        case 64: return pick_c2r_up<64>(up);
        case 128: return pick_c2r_up<128>(up);
    }
    return nullptr;
}

MixKernel pick_mix(int C, int pass) {
    const int C2 = 2 * C;
    if (C == 32) return pass ? fu2d_mix_kernel<2, 1, 32> : fu2d_mix_kernel<2, 0, 32>;   // fgan128 64^2 / 128^2
    if (C == 16) return pass ? fu2d_mix_kernel<1, 1, 16> : fu2d_mix_kernel<1, 0, 16>;
    if (C2 <= 32) return pass ? fu2d_mix_kernel<1, 1> : fu2d_mix_kernel<1, 0>;
    if (C2 <= 64) return pass ? fu2d_mix_kernel<2, 1> : fu2d_mix_kernel<2, 0>;
    if (C2 <= 128) return pass ? fu2d_mix_kernel<4, 1> : fu2d_mix_kernel<4, 0>;
    return nullptr;
}

MixKernel pick_mix16(int C, int pass) {
    if (C == 16) return pass ? fu2d_mix_kernel<1, 1, 16, true> : fu2d_mix_kernel<1, 0, 16, true>;
    if (C == 32) return pass ? fu2d_mix_kernel<2, 1, 32, true> : fu2d_mix_kernel<2, 0, 32, true>;
    if (C == 64) return pass ? fu2d_mix_kernel<4, 1, 64, true> : fu2d_mix_kernel<4, 0, 64, true>;
    return nullptr;
}

// fp16 mix weight [Mpad][2C] (row o = output channel, k contiguous), rows >= 2C zero
__global__ void pack_mix_f16_kernel(const float* __restrict__ w, int C2, int Mpad, _Float16* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= Mpad * C2) return;
    const int o = i / C2;
    out[i] = o < C2 ? (_Float16)w[i] : (_Float16)0.0f;
}

typedef void (*MixKernel2)(MixArgs);
template <int MT, int CC, bool F16>
MixKernel2 pick_cols_h(int H) {
    switch (H) {
        case 32: return fu2d_mix_cols_kernel<MT, CC, F16, 32>;
        case 64: return fu2d_mix_cols_kernel<MT, CC, F16, 64>;
        case 128: return fu2d_mix_cols_kernel<MT, CC, F16, 128>;
    }
    return nullptr;
}
MixKernel2 pick_cols(int C, int H, int f16) {
    if (f16) {
        if (C == 16) return pick_cols_h<1, 16, true>(H);
        if (C == 32) return pick_cols_h<2, 32, true>(H);
        if (C == 64) return pick_cols_h<4, 64, true>(H);
        return nullptr;
    }
    if (C == 16) return pick_cols_h<1, 16, false>(H);
    if (C == 32) return pick_cols_h<2, 32, false>(H);
    return nullptr;
}
size_t cols_lds(int C, int f16) {
    const int Mpad = (2 * C + 31) / 32 * 32;
    const size_t wfl = f16 ? 0 : ((size_t)2 * C * Mpad + 255) / 256 * 256;
    return 4 * (wfl + 4 * (size_t)C) + 8 * (size_t)C * 128 / 32 * 36;   // Ycol: C * CPW * (HC + 4) float2
}
C2rKernel pick_rows(int H, int W, int up) {
    if (H != W) return nullptr;
    switch (H) {
        case 32: return up == 1 ? fu2d_c2r_rows_kernel<32, 32, 1> : fu2d_c2r_rows_kernel<32, 32, 2>;
        case 64: return up == 1 ? fu2d_c2r_rows_kernel<64, 64, 1> : fu2d_c2r_rows_kernel<64, 64, 2>;
        case 128: return up == 1 ? fu2d_c2r_rows_kernel<128, 128, 1> : fu2d_c2r_rows_kernel<128, 128, 2>;
    }
    return nullptr;
}

// + 16 B: the in-kernel BN fold's scale / shift behind the planes
size_t r2c_lds(int h, int w) { return (size_t)h * (w + 4) * 4 + (size_t)h * zstride(w / 2 + 1) * 8 + 16; }
size_t c2r_lds(int H, int W) { return (size_t)H * zstride(W / 2 + 1) * 8 + 16; }
size_t mix_wm_floats(int C) { return (size_t)(2 * C) * ((2 * C + 31) / 32 * 32); }
size_t mix_lds(int C, int pass, bool f16 = false) {
    const size_t wm = f16 ? 0 : (mix_wm_floats(C) + 255) / 256 * 256;   // <= 64 KiB for 2C <= 128
    const size_t tail = pass ? 4 * (size_t)C : (size_t)(FU2_THREADS / 64) * ffc::TILE_SCRATCH;
    return 4 * (wm + tail);
}

int raise_lds(const void* k, size_t lds, const char* what) {
    if (lds <= 64 * 1024) return FFC_OK;
    static std::mutex mu;
    static std::set<const void*> raised;
    std::lock_guard<std::mutex> g(mu);
    if (raised.count(k)) return FFC_OK;
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) {
        ffc::set_error(std::string(what) + ": hipFuncSetAttribute: " + hipGetErrorString(e));
        return FFC_E_LAUNCH;
    }
    raised.insert(k);
    return FFC_OK;
}

// workgroups per sample: ~MIX_TILES_PER_WG bin tiles each (2 per wave), but enough workgroups
// (>= ~1024) to fill the chip when the batch is small, down to one tile per workgroup
int mix_fill_target() {   // FFC_MIX_FILL: workgroups the split aims for at small batches (A/B)
    static const int v = [] {
        const char* e = std::getenv("FFC_MIX_FILL");
        const int n = e ? std::atoi(e) : 0;
        return n > 0 ? n : 512;
    }();
    return v;
}
int mix_nsplit(int B, int H, int W) {
    const int ntiles = (H * (W / 2 + 1) + 31) / 32;
    const int fill = (mix_fill_target() + B - 1) / B;
    return std::max(1, std::min(ntiles, std::max(ntiles / MIX_TILES_PER_WG, fill)));
}

}  // namespace

extern "C" int ffc_fu2d_supported(int C, int H, int W, int up) {
    if (C <= 0 || C > 64 || H != W || !(up == 1 || up == 2)) return 0;   // 2C <= 128
    if (!pow2_in(H, 16, 128)) return 0;
    const int h = H / up;
    if (!pow2_in(h, 8, 128)) return 0;
    if (r2c_lds(h, h) > 160 * 1024 || c2r_lds(H, W) > 160 * 1024) return 0;
    return 1;
}

extern "C" int ffc_fu2d_slab_rows(int B, int C, int H, int W) {
    if (B <= 0 || C <= 0 || H <= 0 || W <= 0) return 0;
    return B * mix_nsplit(B, H, W);
}

extern "C" int ffc_fu2d_r2c(const float* t, int B, int C, int h, int w, const float* in_scale,
                            const float* in_shift, int in_relu, float* T, void* stream) {
    return ffc_fu2d_r2c_ex(t, B, C, h, w, in_scale, in_shift, in_relu, nullptr, T, stream);
}

// a per-channel fold (ffc::bn_fold_channel): momentum >= 0 (no num_batches_tracked read), C channels
static bool channel_fold_ok(const ffc_bn_fold* f, int C) {
    return (f->moments || (f->slab && f->nrows > 0)) && f->C == C && (!f->update_running ||
           (f->running_mean && f->running_var && f->num_batches_tracked && f->momentum >= 0.0f));
}

extern "C" int ffc_fu2d_r2c_ex(const float* t, int B, int C, int h, int w, const float* in_scale,
                               const float* in_shift, int in_relu, const ffc_bn_fold* in_fold, float* T,
                               void* stream) {
    FFC_CHECK_ARG(B > 0 && C > 0, "ffc_fu2d_r2c: B and C must be positive");
    FFC_CHECK_ARG(t && T, "ffc_fu2d_r2c: null pointer");
    FFC_CHECK_ARG((in_scale == nullptr) == (in_shift == nullptr), "ffc_fu2d_r2c: in_scale/in_shift pairing");
    FFC_CHECK_ARG(!in_fold || (!in_scale && channel_fold_ok(in_fold, C) && in_fold->scale_out && in_fold->shift_out),
                  "ffc_fu2d_r2c: in_fold replaces in_scale / in_shift, needs C channels, momentum >= 0 and "
                  "scale_out / shift_out");
    R2cKernel k = pick_r2c(h, w);
    FFC_CHECK_ARG(k != nullptr, "ffc_fu2d_r2c: unsupported plane (square, power of two in [8, 128])");
    const size_t lds = r2c_lds(h, w);
    FFC_CHECK_ARG(lds <= 160 * 1024, "ffc_fu2d_r2c: plane exceeds LDS");
    int rc = raise_lds(reinterpret_cast<const void*>(k), lds, "ffc_fu2d_r2c");
    if (rc) return rc;
    R2cArgs a{t, in_scale, in_shift, T, C, in_relu, 1.0f, 1.0f};
    a.has_fold = in_fold != nullptr;
    if (in_fold) a.fold = *in_fold;
    hipLaunchKernelGGL(k, dim3(B * C), dim3(FU2_THREADS), lds, (hipStream_t)stream, a);
    return ffc::launch_status("ffc_fu2d_r2c");
}

extern "C" int ffc_fu2d_mix(const float* T, int B, int C, int H, int W, int up, const float* wmixT, int pass,
                            float* stats_slab, const float* bn_scale, const float* bn_shift, float* Y,
                            void* stream) {
    FFC_CHECK_ARG(B > 0 && C > 0, "ffc_fu2d_mix: B and C must be positive");
    FFC_CHECK_ARG(ffc_fu2d_supported(C, H, W, up), "ffc_fu2d_mix: unsupported (C, H, W, up)");
    FFC_CHECK_ARG(T && wmixT, "ffc_fu2d_mix: null pointer");
    FFC_CHECK_ARG(pass == 0 || pass == 1, "ffc_fu2d_mix: pass must be 0 or 1");
    if (pass == 0) FFC_CHECK_ARG(stats_slab != nullptr, "ffc_fu2d_mix: pass 0 needs stats_slab");
    if (pass == 1) FFC_CHECK_ARG(bn_scale && bn_shift && Y, "ffc_fu2d_mix: pass 1 needs bn_scale/shift/Y");
    MixKernel k = pick_mix(C, pass);
    FFC_CHECK_ARG(k != nullptr, "ffc_fu2d_mix: 2C > 128");
    MixArgs a;
    a.T = T;
    a.wmixT = wmixT;
    a.slab = stats_slab;
    a.bn_scale = bn_scale;
    a.bn_shift = bn_shift;
    a.Y = Y;
    a.B = B;
    a.C = C;
    a.H = H;
    a.W = W;
    a.up = up;
    a.ntiles = (H * (W / 2 + 1) + 31) / 32;
    a.nsplit = mix_nsplit(B, H, W);
    a.Mpad = (2 * C + 31) / 32 * 32;
    a.norm = (float)(1.0 / std::sqrt((double)H * (double)W));
    const size_t lds = mix_lds(C, pass);
    int rc = raise_lds(reinterpret_cast<const void*>(k), lds, "ffc_fu2d_mix");
    if (rc) return rc;
    hipLaunchKernelGGL(k, dim3(B * a.nsplit), dim3(FU2_THREADS), lds, (hipStream_t)stream, a);
    return ffc::launch_status("ffc_fu2d_mix");
}

namespace {
typedef void (*R2cMixKernel)(R2cMixArgs);
R2cMixKernel pick_r2c_mix(int C, int h, size_t& lds) {
    if (C == 16 && h == 8) return lds = 4 * R2cMixLds<8, 16>::FLOATS, fu2d_r2c_mix_kernel<1, 16, 8>;
    if (C == 16 && h == 16) return lds = 4 * R2cMixLds<16, 16>::FLOATS, fu2d_r2c_mix_kernel<1, 16, 16>;
    if (C == 32 && h == 8) return lds = 4 * R2cMixLds<8, 32>::FLOATS, fu2d_r2c_mix_kernel<2, 32, 8>;
    if (C == 32 && h == 16) return lds = 4 * R2cMixLds<16, 32>::FLOATS, fu2d_r2c_mix_kernel<2, 32, 16>;
    return nullptr;
}
}  // namespace

#ifdef FFC_R2CMIX_DUMP
extern "C" int ffc_debug_r2cmix_dump(void* dst, size_t bytes) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_r2cmix_dump), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
#if defined(FFC_R2CMIX_DBG) || defined(FFC_R2CMIX_DBGEND)
extern "C" int ffc_debug_r2cmix_read(void* dst, size_t bytes) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_r2cmix_dbg), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int ffc_fu2d_r2c_mix_supported(int C, int H, int W, int up) {
    size_t lds = 0;
    return ffc_fu2d_supported(C, H, W, up) && pick_r2c_mix(C, H / up, lds) != nullptr && lds <= 160 * 1024;
}

extern "C" int ffc_fu2d_r2c_mix(const float* t, int B, int C, int H, int W, int up, const float* in_scale,
                                const float* in_shift, int in_relu, const ffc_bn_fold* in_fold, const float* wmixT,
                                float* stats_slab, float* Y, void* stream) {
    FFC_CHECK_ARG(B > 0 && C > 0, "ffc_fu2d_r2c_mix: B and C must be positive");
    FFC_CHECK_ARG(ffc_fu2d_r2c_mix_supported(C, H, W, up), "ffc_fu2d_r2c_mix: unsupported (C, H, W, up)");
    FFC_CHECK_ARG(t && wmixT && stats_slab && Y, "ffc_fu2d_r2c_mix: null pointer");
    FFC_CHECK_ARG((in_scale == nullptr) == (in_shift == nullptr), "ffc_fu2d_r2c_mix: in_scale/in_shift pairing");
    FFC_CHECK_ARG(!in_fold || (!in_scale && channel_fold_ok(in_fold, C) && in_fold->scale_out && in_fold->shift_out),
                  "ffc_fu2d_r2c_mix: in_fold replaces in_scale / in_shift, needs C channels, momentum >= 0 and "
                  "scale_out / shift_out");
    size_t lds = 0;
    R2cMixKernel k = pick_r2c_mix(C, H / up, lds);
#ifdef FFC_R2CMIX_ONEWG   // DESIGN 10c probe: a dynamic LDS request that admits one workgroup per CU
    lds = 90 * 1024;
#endif
#ifdef FFC_R2CMIX_PAD     // DESIGN 10c probe: unused LDS behind the layout, still two workgroups per CU
    lds += FFC_R2CMIX_PAD;
#endif
#ifdef FFC_R2CMIX_FRONTPAD
    lds += FFC_R2CMIX_FRONTPAD;
#endif
    int rc = raise_lds(reinterpret_cast<const void*>(k), lds, "ffc_fu2d_r2c_mix");
    if (rc) return rc;
    R2cMixArgs ra;
    MixArgs& a = ra.m;
    a.T = nullptr;
    a.wmixT = wmixT;
    a.slab = stats_slab;
    a.bn_scale = nullptr;
    a.bn_shift = nullptr;
    a.Y = Y;
    a.B = B;
    a.C = C;
    a.H = H;
    a.W = W;
    a.up = up;
    a.ntiles = (H * (W / 2 + 1) + 31) / 32;
    a.nsplit = mix_nsplit(B, H, W);   // the slab rows of ffc_fu2d_slab_rows
    a.Mpad = (2 * C + 31) / 32 * 32;
    a.norm = (float)(1.0 / std::sqrt((double)H * (double)W));
    ra.t = t;
    ra.in_scale = in_scale;
    ra.in_shift = in_shift;
    ra.in_relu = in_relu;
    ra.has_fold = in_fold != nullptr;
    if (in_fold) ra.fold = *in_fold;
    hipLaunchKernelGGL(k, dim3(B * a.nsplit), dim3(FU2_THREADS), lds, (hipStream_t)stream, ra);
    return ffc::launch_status("ffc_fu2d_r2c_mix");
}

extern "C" int ffc_fu_pack_mix_f16(const float* w, int C2, void* w16, void* stream) {
    FFC_CHECK_ARG(w && w16 && C2 > 0, "ffc_fu_pack_mix_f16: bad args");
    const int Mpad = (C2 + 31) / 32 * 32;
    const int n = Mpad * C2;
    hipLaunchKernelGGL(pack_mix_f16_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, w, C2, Mpad,
                       reinterpret_cast<_Float16*>(w16));
    return ffc::launch_status("ffc_fu_pack_mix_f16");
}

extern "C" int ffc_fu2d_mix_f16(const float* T, int B, int C, int H, int W, int up, const void* wmix16, int pass,
                                float* stats_slab, const float* bn_scale, const float* bn_shift, float* Y,
                                void* stream) {
    FFC_CHECK_ARG(B > 0 && C > 0, "ffc_fu2d_mix_f16: B and C must be positive");
    FFC_CHECK_ARG(ffc_fu2d_supported(C, H, W, up), "ffc_fu2d_mix_f16: unsupported (C, H, W, up)");
    FFC_CHECK_ARG(T && wmix16, "ffc_fu2d_mix_f16: null pointer");
    FFC_CHECK_ARG(pass == 0 || pass == 1, "ffc_fu2d_mix_f16: pass must be 0 or 1");
    if (pass == 0) FFC_CHECK_ARG(stats_slab != nullptr, "ffc_fu2d_mix_f16: pass 0 needs stats_slab");
    if (pass == 1) FFC_CHECK_ARG(bn_scale && bn_shift && Y, "ffc_fu2d_mix_f16: pass 1 needs bn_scale/shift/Y");
    MixKernel k = pick_mix16(C, pass);
    FFC_CHECK_ARG(k != nullptr, "ffc_fu2d_mix_f16: C must be 16, 32 or 64");
    MixArgs a;
    a.T = T;
    a.wmixT = reinterpret_cast<const float*>(wmix16);
    a.slab = stats_slab;
    a.bn_scale = bn_scale;
    a.bn_shift = bn_shift;
    a.Y = Y;
    a.B = B;
    a.C = C;
    a.H = H;
    a.W = W;
    a.up = up;
    a.ntiles = (H * (W / 2 + 1) + 31) / 32;
    a.nsplit = mix_nsplit(B, H, W);
    a.Mpad = (2 * C + 31) / 32 * 32;
    a.norm = (float)(1.0 / std::sqrt((double)H * (double)W));
    const size_t lds = mix_lds(C, pass, true);
    hipLaunchKernelGGL(k, dim3(B * a.nsplit), dim3(FU2_THREADS), lds, (hipStream_t)stream, a);
    return ffc::launch_status("ffc_fu2d_mix_f16");
}

static int fu2d_c2r_launch(const float* Y, int B, int C, int H, int W, const float* t, int up,
                           const float* in_scale, const float* in_shift, int in_relu, int residual,
                           const float* bn_scale, const float* bn_shift, float* out, void* stream,
                           const ffc_bn_fold* bn_fold = nullptr) {
    FFC_CHECK_ARG(B > 0 && C > 0, "ffc_fu2d_c2r: B and C must be positive");
    FFC_CHECK_ARG((bn_scale == nullptr) == (bn_shift == nullptr), "ffc_fu2d_c2r: bn_scale/bn_shift pairing");
    FFC_CHECK_ARG(Y && out, "ffc_fu2d_c2r: null pointer");
    FFC_CHECK_ARG(!residual || t, "ffc_fu2d_c2r: residual needs t");
    FFC_CHECK_ARG(up == 1 || up == 2, "ffc_fu2d_c2r: up must be 1 or 2");
    FFC_CHECK_ARG((in_scale == nullptr) == (in_shift == nullptr), "ffc_fu2d_c2r: in_scale/in_shift pairing");
    C2rArgs a{Y, t, in_scale, in_shift, out, C, in_relu, residual, (float)(1.0 / std::sqrt((double)H * (double)W)),
              bn_scale, bn_shift, 1.0f};
    a.has_bn_fold = bn_fold != nullptr;
    if (bn_fold) a.bn_fold = *bn_fold;
    C2rKernel k = pick_c2r(H, W, up);
    FFC_CHECK_ARG(k != nullptr, "ffc_fu2d_c2r: unsupported plane (square, power of two in [16, 128])");
    const size_t lds = c2r_lds(H, W);
    int rc = raise_lds(reinterpret_cast<const void*>(k), lds, "ffc_fu2d_c2r");
    if (rc) return rc;
    hipLaunchKernelGGL(k, dim3(B * C), dim3(FU2_THREADS), lds, (hipStream_t)stream, a);
    return ffc::launch_status("ffc_fu2d_c2r");
}

extern "C" int ffc_fu2d_c2r(const float* Y, int B, int C, int H, int W, const float* t, int up,
                            const float* in_scale, const float* in_shift, int in_relu, int residual, float* out,
                            void* stream) {
    return fu2d_c2r_launch(Y, B, C, H, W, t, up, in_scale, in_shift, in_relu, residual, nullptr, nullptr, out,
                           stream);
}

extern "C" int ffc_fu2d_c2r_bn(const float* Y, int B, int C, int H, int W, const float* t, int up,
                               const float* in_scale, const float* in_shift, int in_relu, int residual,
                               const float* bn_scale, const float* bn_shift, float* out, void* stream) {
    FFC_CHECK_ARG(bn_scale && bn_shift, "ffc_fu2d_c2r_bn: bn_scale and bn_shift required");
    return fu2d_c2r_launch(Y, B, C, H, W, t, up, in_scale, in_shift, in_relu, residual, bn_scale, bn_shift, out,
                           stream);
}

extern "C" int ffc_fu2d_c2r_fold(const float* Y, int B, int C, int H, int W, const float* t, int up,
                                 const float* in_scale, const float* in_shift, int in_relu, int residual,
                                 const ffc_bn_fold* bn_fold, float* out, void* stream) {
    FFC_CHECK_ARG(bn_fold && channel_fold_ok(bn_fold, 2 * C),
                  "ffc_fu2d_c2r_fold: bn_fold needs 2C channels and momentum >= 0");
    return fu2d_c2r_launch(Y, B, C, H, W, t, up, in_scale, in_shift, in_relu, residual, nullptr, nullptr, out,
                           stream, bn_fold);
}

extern "C" int ffc_fu2d_cols_supported(int C, int H, int W, int up, int f16) {
    if (!ffc_fu2d_supported(C, H, W, up) || !pick_cols(C, H, f16) || !pick_rows(H, W, up)) return 0;
    return cols_lds(C, f16) <= 160 * 1024;
}

extern "C" int ffc_fu2d_mix_cols(const float* T, int B, int C, int H, int W, int up, const void* wmix, int f16,
                                 const float* bn_scale, const float* bn_shift, float* Yc, void* stream) {
    FFC_CHECK_ARG(B > 0 && T && wmix && bn_scale && bn_shift && Yc, "ffc_fu2d_mix_cols: bad args");
    FFC_CHECK_ARG(ffc_fu2d_cols_supported(C, H, W, up, f16), "ffc_fu2d_mix_cols: unsupported (C, H, W, up)");
    MixKernel2 k = pick_cols(C, H, f16);
    MixArgs a;
    a.T = T;
    a.wmixT = reinterpret_cast<const float*>(wmix);
    a.slab = nullptr;
    a.bn_scale = bn_scale;
    a.bn_shift = bn_shift;
    a.Y = Yc;
    a.B = B;
    a.C = C;
    a.H = H;
    a.W = W;
    a.up = up;
    a.ntiles = 0;
    a.Mpad = (2 * C + 31) / 32 * 32;
    a.norm = (float)(1.0 / std::sqrt((double)H * (double)W));
    const size_t lds = cols_lds(C, f16);
    int rc = raise_lds(reinterpret_cast<const void*>(k), lds, "ffc_fu2d_mix_cols");
    if (rc) return rc;
    const int cpw = 4 / (H / 32);
    const int ncg = (W / 2 + 1 + cpw - 1) / cpw;
    // ~4 column groups per workgroup, but >= ~512 workgroups in all
    a.nsplit = std::max(1, std::min(ncg, std::max(ncg / 4, (512 + B - 1) / B)));
    hipLaunchKernelGGL(k, dim3(B * a.nsplit), dim3(FU2_THREADS), lds, (hipStream_t)stream, a);
    return ffc::launch_status("ffc_fu2d_mix_cols");
}

extern "C" int ffc_fu2d_c2r_rows(const float* Yc, int B, int C, int H, int W, const float* t, int up,
                                 const float* in_scale, const float* in_shift, int in_relu, int residual, float* out,
                                 void* stream) {
    FFC_CHECK_ARG(B > 0 && C > 0 && Yc && out, "ffc_fu2d_c2r_rows: bad args");
    FFC_CHECK_ARG(!residual || t, "ffc_fu2d_c2r_rows: residual needs t");
    FFC_CHECK_ARG((in_scale == nullptr) == (in_shift == nullptr), "ffc_fu2d_c2r_rows: in_scale/in_shift pairing");
    C2rKernel k = pick_rows(H, W, up);
    FFC_CHECK_ARG(k != nullptr, "ffc_fu2d_c2r_rows: unsupported plane (square, 32..128)");
    const int RB = H < 64 ? H : 64;
    const size_t lds = (size_t)RB * zstride(W / 2 + 1) * 8;
    C2rArgs a{Yc, t, in_scale, in_shift, out, C, in_relu, residual, (float)(1.0 / std::sqrt((double)H * (double)W)),
              nullptr, nullptr, 1.0f};
    hipLaunchKernelGGL(k, dim3(B * C * (H / RB)), dim3(FU2_THREADS), lds, (hipStream_t)stream, a);
    return ffc::launch_status("ffc_fu2d_c2r_rows");
}

// ---- the training path's planar transforms (ffc_rfft2_planes / ffc_irfft2_planes, train_kernels.hip)
// on the line FFTs above: square power-of-two planes 8..128 (r2c) / 16..128 (c2r); 0 = handled,
// 1 = not supported here (the caller falls back to its direct DFT, planes <= 64).
namespace {
template <int N>
R2cKernel pick_r2c_planar_n() { return fu2d_r2c_kernel<N, N, true>; }
R2cKernel pick_r2c_planar(int H, int W) {
    if (H != W) return nullptr;
    switch (H) {
        case 8: return pick_r2c_planar_n<8>();
        case 16: return pick_r2c_planar_n<16>();
        case 32: return pick_r2c_planar_n<32>();
        case 64: return pick_r2c_planar_n<64>();
        case 128: return pick_r2c_planar_n<128>();
    }
    return nullptr;
}
C2rKernel pick_c2r_planar(int H, int W) {
    if (H != W) return nullptr;
    switch (H) {
        case 16: return fu2d_c2r_kernel<16, 16, 1, true>;
        case 32: return fu2d_c2r_kernel<32, 32, 1, true>;
        case 64: return fu2d_c2r_kernel<64, 64, 1, true>;
        case 128: return fu2d_c2r_kernel<128, 128, 1, true>;
    }
    return nullptr;
}
}  // namespace

namespace ffc {
int fft_planes_r2c(const float* x, int P, int H, int W, float iscale, float* Z, void* stream) {
    R2cKernel k = pick_r2c_planar(H, W);
    if (!k) return 1;
    const size_t lds = r2c_lds(H, W);
    if (lds > 160 * 1024) return 1;
    int rc = raise_lds(reinterpret_cast<const void*>(k), lds, "ffc_rfft2_planes");
    if (rc) return rc;
    R2cArgs a{x, nullptr, nullptr, Z, 1, 0, (float)(1.0 / std::sqrt((double)H * (double)W)), iscale};
    hipLaunchKernelGGL(k, dim3(P), dim3(FU2_THREADS), lds, (hipStream_t)stream, a);
    return launch_status("ffc_rfft2_planes");
}

int fft_planes_c2r(const float* Z, int P, int H, int W, float iscale, const float* addend, float* y, void* stream) {
    C2rKernel k = pick_c2r_planar(H, W);
    if (!k) return 1;
    const size_t lds = c2r_lds(H, W);
    if (lds > 160 * 1024) return 1;
    int rc = raise_lds(reinterpret_cast<const void*>(k), lds, "ffc_irfft2_planes");
    if (rc) return rc;
    C2rArgs a{Z, addend, nullptr, nullptr, y, 1, 0, addend ? 1 : 0,
              (float)(1.0 / std::sqrt((double)H * (double)W)), nullptr, nullptr, iscale};
    hipLaunchKernelGGL(k, dim3(P), dim3(FU2_THREADS), lds, (hipStream_t)stream, a);
    return launch_status("ffc_irfft2_planes");
}
}  // namespace ffc
