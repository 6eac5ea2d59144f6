// Fused Fourier unit for gfx950: one workgroup (8 waves) per sample.
//
// Replaces FourierUnitSN.forward (layers/ffc/fourier_unity.py:32-56) and, through the
// input transform, the bn1/act1/Upsample prologue of SpectralTransform.forward
// (layers/ffc/spectral_transform.py:79-91) plus the residual add of :108.
//
//   HBM  --row loads-->  regs: real W-point FFT per (channel,row)  --> LDS Z planes (Re, Im)
//   LDS  column H-point FFT per (channel, k_w), ortho scale            (in place)
//   LDS  spectral mix  Y = Wmix . Z  on v_mfma_f32_32x32x2_f32 (exact fp32), K = 2C
//        pass 0: per-tile Chan partials of Y -> one {n, mean, M2} per channel -> HBM slab
//        pass 1: BN scale/shift + ReLU -> LDS Y planes
//   LDS  inverse column FFT; per-row C2R (Im of k_w = 0, W/2 ignored) + residual --> HBM
//
// Train-mode BN needs batch statistics between the mix and its apply; the kernel is run
// twice (pass 0 then pass 1) and recomputes the cheap FFT+mix instead of spilling Y to HBM,
// so a train-mode FU moves 2 reads + 1 write of the activation (SURVEY.md §8d "12*N_r").
#include "ffc_internal.h"
#include "bn_common.h"

#include <cmath>
#include <cstdlib>
#include <mutex>
#include <set>

#include "fft_common.h"

namespace {

template <int N>
__device__ __forceinline__ void load_row(const float* __restrict__ p, float (&v)[N]) {
    if constexpr (N % 4 == 0) {
#pragma unroll
        for (int i = 0; i < N / 4; ++i) {
            const float4 q = reinterpret_cast<const float4*>(p)[i];
            v[4 * i] = q.x; v[4 * i + 1] = q.y; v[4 * i + 2] = q.z; v[4 * i + 3] = q.w;
        }
    } else if constexpr (N % 2 == 0) {
#pragma unroll
        for (int i = 0; i < N / 2; ++i) {
            const float2 q = reinterpret_cast<const float2*>(p)[i];
            v[2 * i] = q.x; v[2 * i + 1] = q.y;
        }
    } else {
#pragma unroll
        for (int i = 0; i < N; ++i) v[i] = p[i];
    }
}

template <int N>
__device__ __forceinline__ void store_row(float* __restrict__ p, const float (&v)[N]) {
    static_assert(N % 4 == 0, "rows are >= 4 wide");
#pragma unroll
    for (int i = 0; i < N / 4; ++i)
        reinterpret_cast<float4*>(p)[i] = make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
}

struct FuArgs {
    const float* t;
    const float* in_scale;
    const float* in_shift;
    const float* wmixT;
    float* slab;
    const float* bn_scale;
    const float* bn_shift;
    float* out;
    int C, Mpad, in_relu, residual, has_in_affine;
    int wm_lds;   // mix weight staged in LDS (when it fits beside the Z/Y planes)
    int scr_off;  // float offset of the pass-0 stats scratch in LDS
    int bn_off;   // float offset of the pass-1 BN scale/shift (4C floats), then the folded input affine (2C)
    float norm;
    ffc_bn_fold in_fold, mix_fold;   // BNs finalized in-kernel (has_*: in use)
    int has_in_fold, has_mix_fold;
    float* yspill;                   // (B, 2C, NB) mix output: written by pass 0, read by pass 1
    int mix3;                        // mix on split-bf16 MFMA products (C % 8 == 0), else f32-input MFMA
    const uint16_t* wmix3;           // mix weight pre-split in fragment order (ffc_fu_pack_mix3), or null
    int w3_lds;                      // wmix3 staged in the LDS weight region instead of wmixT
    int mgroups;                     // pass 0: workgroups per sample, each mixing MT / mgroups M-tiles
    int B;
    int kgroups;                     // bin groups of pass 0 (fu_pass0_kg_kernel): slab rows, spill layout
    int shuf;                        // column DFTs across lanes (fft_common.h lane_fft_dif / lane_ifft_dit)
};

constexpr int FU_THREADS = 512;

// floats of the LDS mix-weight region: (2C, ceil32(2C)) in whole 64-lane x 16-B DMA groups
__host__ __device__ inline size_t fu_wm_floats(int C) {
    const size_t Mpad = (size_t)(2 * C + 31) / 32 * 32;
    return ((size_t)(2 * C) * Mpad + 255) / 256 * 256;
}
// Pass-0 per-wave stats scratch (FuArgs::scr_off): the Y-imaginary plane (unused in pass 0)
// when it is large enough, else a region after the planes (and the mix weight, when staged).
constexpr int FU_SCRATCH = (FU_THREADS / 64) * 32 * 33;

#ifdef FFC_TRACE
// Diagnostic build only: per workgroup {realtime start, end, s_memtime at phase boundaries 0..5}.
__device__ unsigned long long g_fu_trace[8 * 4096];
#define FU_STAMP(i)                                                                         \
    do {                                                                                    \
        unsigned long long t_;                                                              \
        __builtin_amdgcn_sched_barrier(0);                                                  \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");         \
        __builtin_amdgcn_sched_barrier(0);                                                  \
        if (threadIdx.x == 0) g_fu_trace[8 * blockIdx.x + 2 + (i)] = t_;                   \
    } while (0)
#else
#define FU_STAMP(i) do { } while (0)
#endif

// s row (channel ch, output row y) = transform(t) nearest-upsampled by UP; the input affine from
// LDS (folded in this kernel) or global memory
template <int W, int UP>
__device__ __forceinline__ void load_s_row(const FuArgs& a, const float* insc, int b, int ch, int y, int H,
                                           float (&s)[W]) {
    constexpr int tW = W / UP;
    const int tH = H / UP;
    const float* trow = a.t + ((size_t)(b * a.C + ch) * tH + y / UP) * tW;
    float tv[tW];
    load_row<tW>(trow, tv);
    float sc = 1.0f, sh = 0.0f;
    if (a.has_in_fold) {
        sc = insc[ch];
        sh = insc[a.C + ch];
    } else if (a.has_in_affine) {
        sc = a.in_scale[ch];
        sh = a.in_shift[ch];
    }
#pragma unroll
    for (int x = 0; x < W; ++x) {
        float v = tv[x / UP];
        v = fmaf(v, sc, sh);
        if (a.in_relu) v = fmaxf(v, 0.0f);
        s[x] = v;
    }
}

// bin groups of the fused FU's pass 0 (fu_pass0_kg_kernel below): columns per group
template <int W, int G>
struct FuKg {
    static constexpr int WP = W / 2 + 1;
    static constexpr int KW0 = (WP + G - 1) / G;
    static constexpr int KWL = WP - (G - 1) * KW0;   // the last group's columns
    static_assert(KWL >= 1, "every bin group non-empty");
};

// spill offset (within a channel's NB floats) of bin (y, k) -> the natural bin index y WP + k:
// the inverse map pass 1 applies to the bin-group layout
template <int H, int W, int G>
__device__ __forceinline__ int fu_spill_bin(int m) {
    if constexpr (G == 1) {
        return m;
    } else {
        using K = FuKg<W, G>;
        constexpr int ZPL = H * K::KW0;
        const int g = min(m / ZPL, G - 1);
        const int rem = m - g * ZPL;
        const int y = g < G - 1 ? rem / K::KW0 : rem / K::KWL;
        const int kk = rem - y * (g < G - 1 ? K::KW0 : K::KWL);
        return y * K::WP + g * K::KW0 + kk;
    }
}

// BN + ReLU of spilled floats m .. m + 3 of one channel -> its Y plane (natural bin order)
template <int H, int W, int G>
__device__ __forceinline__ void spill_to_plane(float* dst, int m, float4 v, float sc, float sh) {
    v = make_float4(fmaxf(fmaf(v.x, sc, sh), 0.0f), fmaxf(fmaf(v.y, sc, sh), 0.0f), fmaxf(fmaf(v.z, sc, sh), 0.0f),
                    fmaxf(fmaf(v.w, sc, sh), 0.0f));
    if constexpr (G == 1) {
        *reinterpret_cast<float4*>(dst + m) = v;
    } else {
        dst[fu_spill_bin<H, W, G>(m)] = v.x;
        dst[fu_spill_bin<H, W, G>(m + 1)] = v.y;
        dst[fu_spill_bin<H, W, G>(m + 2)] = v.z;
        dst[fu_spill_bin<H, W, G>(m + 3)] = v.w;
    }
}

template <int H, int W, int UP, int PASS>
__global__ __launch_bounds__(FU_THREADS) void fu_kernel(FuArgs a) {
    constexpr int WP = W / 2 + 1;
    constexpr int NB = H * WP;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int C = a.C;
    const int C2 = 2 * C;
    // pass 0 over mgroups workgroups per sample (small batches: more CUs): each repeats the sample's
    // FFTs and mixes / spills / reduces the statistics of its own M-tiles only
    const int G = PASS == 0 ? a.mgroups : 1;
    const int b = blockIdx.x / G, grp = blockIdx.x - b * G;
    const int tid = threadIdx.x;
    float* Zre = smem;
    float* Zim = Zre + C * NB;
    float* Yre = Zim + C * NB;
    float* Yim = Yre + C * NB;
    float* Wm = Yim + C * NB;   // mix weight (2C, Mpad), staged by LDS-DMA under the FFT phases
    const bool from_spill = PASS == 1 && a.yspill != nullptr;   // pass 1 without the recompute
    if (a.wm_lds && !from_spill) {
        typedef __attribute__((address_space(1))) void* gptr_t;
        typedef __attribute__((address_space(3))) void* lptr_t;
        // the f32 weight (2C x Mpad floats) or its split pieces (Mpad / 32 x C / 8 fragments of 3 KB)
        const float* wsrc = a.w3_lds ? reinterpret_cast<const float*>(a.wmix3) : a.wmixT;
        const int n4 = a.w3_lds ? (a.Mpad >> 5) * (C >> 3) * 192 : (C2 * a.Mpad) >> 2;   // 16-byte groups
        for (int i0 = 0; i0 < n4; i0 += FU_THREADS) {
            if (i0 + (tid & ~63) < n4) {   // whole wave-instructions; the region is padded to 64 groups
                const int i = min(i0 + tid, n4 - 1);
                __builtin_amdgcn_global_load_lds((gptr_t)(wsrc + 4 * (size_t)i),
                                                 (lptr_t)(Wm + 4 * (i0 + (tid & ~63))), 16, 0, 0);
            }
        }
    }
#ifdef FFC_TRACE
    if (tid == 0) g_fu_trace[8 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
#endif
    FU_STAMP(0);
    const int lane = tid & 63, wave = tid >> 6, h = lane >> 5, col = lane & 31;
    const int MT = (C2 + 31) >> 5, NTL = (NB + 31) >> 5;
    const int MTG = MT / G;   // this workgroup's M-tiles (pass 0): grp * MTG .. grp * MTG + MTG - 1
    float* bnss = smem + a.bn_off;    // pass 1: BN scale [2C] | shift [2C]
    float* insc = bnss + 2 * C2;      // folded input affine: scale [C] | shift [C]
    // fold scratch: the Z/Y planes, all free until the row R2C / spill load below
    double* fscr = reinterpret_cast<double*>(smem);
    if (a.has_in_fold) ffc::bn_fold_block<FU_THREADS>(a.in_fold, insc, insc + C, blockIdx.x == 0, fscr);
    if constexpr (PASS == 1) {
        if (a.has_mix_fold) {
            ffc::bn_fold_block<FU_THREADS>(a.mix_fold, bnss, bnss + C2, blockIdx.x == 0, fscr);
        } else {
            for (int i = tid; i < C2; i += FU_THREADS) {
                bnss[i] = a.bn_scale[i];
                bnss[C2 + i] = a.bn_shift[i];
            }
        }
    }
    if (from_spill) {
        // Y of this sample from pass 0 -> BN + ReLU -> the Y planes (float4: NB is a multiple of 4)
        __syncthreads();
        const float4* ys = reinterpret_cast<const float4*>(a.yspill + (size_t)b * C2 * NB);
        for (int i = tid; i < C2 * NB / 4; i += FU_THREADS) {
            const int o = (4 * i) / NB, n = 4 * i - o * NB;
            const float4 v = ys[i];
            const float sc = bnss[o], sh = bnss[C2 + o];
            float* dst = ((o & 1) ? Yim : Yre) + (o >> 1) * NB;
            if (a.kgroups == 2)
                spill_to_plane<H, W, 2>(dst, n, v, sc, sh);
            else
                spill_to_plane<H, W, 1>(dst, n, v, sc, sh);
        }
        __syncthreads();
    } else {

    if (a.shuf) {
        // 1+2. row R2C in registers, then the column DFTs across the H lanes that hold the channel's
        //      rows (lane_fft_dif: DPP / ds_swizzle butterfly exchanges, ortho scale folded in): no LDS
        //      round trip and no barrier between the row and column transforms.  Lane y ends with
        //      spectrum row bitrev(y), stored to its natural place.
        for (int r = tid; r < C * H; r += FU_THREADS) {
            const int ch = r / H, y = r - ch * H;
            float sv[W], re[WP], im[WP];
            load_s_row<W, UP>(a, insc, b, ch, y, H, sv);
            rfft_reg<W>(sv, re, im);
            lane_fft_dif<H, WP>(re, im, y, a.norm);
            const int yo = lane_brev<H>(y);
            float* zr = Zre + (ch * H + yo) * WP;
            float* zi = Zim + (ch * H + yo) * WP;
#pragma unroll
            for (int k = 0; k < WP; ++k) {
                zr[k] = re[k];
                zi[k] = im[k];
            }
        }
        FU_STAMP(1);
        if (a.wm_lds) ffc::dma_wait();
        __syncthreads();
        FU_STAMP(2);
    } else {
    // 1. row R2C (real W-point FFT per (channel,row) on a W/2-point complex FFT), input transform fused
    for (int r = tid; r < C * H; r += FU_THREADS) {
        const int ch = r / H, y = r - ch * H;
        float sv[W], re[WP], im[WP];
        load_s_row<W, UP>(a, insc, b, ch, y, H, sv);
        rfft_reg<W>(sv, re, im);
        float* zr = Zre + (ch * H + y) * WP;
        float* zi = Zim + (ch * H + y) * WP;
#pragma unroll
        for (int k = 0; k < WP; ++k) {
            zr[k] = re[k];
            zi[k] = im[k];
        }
    }
    FU_STAMP(1);
    if (a.wm_lds) ffc::dma_wait();   // the weight's LDS-DMA retired before the barrier (ffc_internal.h)
    __syncthreads();

    // 2. column C2C over H, ortho scale 1/sqrt(HW)
    for (int q = tid; q < C * WP; q += FU_THREADS) {
        const int ch = q / WP, k = q - ch * WP;
        float* zr = Zre + ch * NB + k;
        float* zi = Zim + ch * NB + k;
        float re[H], im[H];
#pragma unroll
        for (int y = 0; y < H; ++y) {
            re[y] = zr[y * WP];
            im[y] = zi[y * WP];
        }
        fft_reg<H, false>(re, im);
#pragma unroll
        for (int y = 0; y < H; ++y) {
            zr[y * WP] = re[y] * a.norm;
            zi[y * WP] = im[y] * a.norm;
        }
    }
    __syncthreads();
    FU_STAMP(2);
    }   // !a.shuf

    // 3. spectral mix on MFMA: Y[o][n] = sum_i Wmix[o][i] Z[i][n], Z[2c+h] = (h ? Im : Re)(channel c)
    //    k-step s feeds k-slot h = lane>>5 with channel s, component h.
    for (int tile = wave; tile < MTG * NTL; tile += FU_THREADS / 64) {
        const int mt = grp * MTG + tile % MTG, nt = tile / MTG;
        floatx16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
        const float* zp = (h ? Zim : Zre) + nt * 32 + col;
        const int wstep = 2 * a.Mpad;
        if (a.mix3 && a.wmix3) {
            // the weight's pieces come pre-split (ffc_fu_pack_mix3: one 16-byte read per piece and
            // k-block); only Z is split here
            const int QN = C >> 3;
            const uint16_t* w3 = (a.w3_lds ? reinterpret_cast<const uint16_t*>(Wm) : a.wmix3) +
                                 (size_t)mt * QN * 1536 + lane * 8;
#pragma unroll 2
            for (int q = 0; q < QN; ++q) {
                Split3 av;
                av.hi = *reinterpret_cast<const bf16x8*>(w3 + q * 1536);
                av.mid = *reinterpret_cast<const bf16x8*>(w3 + q * 1536 + 512);
                av.lo = *reinterpret_cast<const bf16x8*>(w3 + q * 1536 + 1024);
                float zv[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) zv[j] = zp[(8 * q + j) * NB];
                acc = mfma_split3(av, split3(zv), acc);
            }
        } else if (a.mix3) {
            // fp32-accurate split-bf16 products (ffc_internal.h split3 / mfma_split3): k-block q, lane
            // half h element j is k = 2 (8q + j) + h -- channel 8q + j, Re (h = 0) or Im (h = 1) --
            // in both operands; six bf16 MFMAs per 16 k instead of eight f32 MFMAs at twice the cycles
            const float* wsrc = a.wm_lds ? Wm : a.wmixT;
            const float* wq = wsrc + h * a.Mpad + mt * 32 + col;
#pragma unroll 2
            for (int q = 0; q < C / 8; ++q) {
                float av[8], zv[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    av[j] = wq[(size_t)(8 * q + j) * wstep];
                    zv[j] = zp[(8 * q + j) * NB];
                }
                acc = mfma_split3(split3(av), split3(zv), acc);
            }
        } else if (a.wm_lds) {
            const float* wp = Wm + h * a.Mpad + mt * 32 + col;
#pragma unroll 8
            for (int s = 0; s < C; ++s)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wp[s * wstep], zp[s * NB], acc, 0, 0, 0);
        } else {
            const float* __restrict__ wp = a.wmixT + h * a.Mpad + mt * 32 + col;
#pragma unroll 8
            for (int s = 0; s < C; ++s)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wp[(size_t)s * wstep], zp[s * NB], acc, 0, 0, 0);
        }
        const int n = nt * 32 + col;
        const bool nvalid = n < NB;
        if constexpr (PASS == 0) {
            if (a.yspill) {   // raw Y for pass 1 (row o: 32 consecutive bins per store)
                float* ys = a.yspill + (size_t)b * C2 * NB;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int o = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    if (nvalid && o < C2) ys[(size_t)o * NB + n] = acc[r];
                }
            }
            const int nv = min(32, NB - nt * 32);
            float mean, m2;
            ffc::tile_row_stats(acc, nv, smem + a.scr_off + wave * ffc::TILE_SCRATCH, mean, m2);
            const int o = mt * 32 + (lane >> 1);
            if ((lane & 1) == 0 && o < C2) {
                float* st = Yre + (nt * C2 + o) * 3;
                st[0] = (float)nv;
                st[1] = mean;
                st[2] = m2;
            }
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int o = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (nvalid && o < C2) {
                    const float v = fmaxf(fmaf(acc[r], bnss[o], bnss[C2 + o]), 0.0f);
                    ((o & 1) ? Yim : Yre)[(o >> 1) * NB + n] = v;
                }
            }
        }
    }
    __syncthreads();
    FU_STAMP(3);
    }   // !from_spill

    if constexpr (PASS == 0) {
        FU_STAMP(4);
        // merge the per-tile partials of each channel (Chan et al.) -> one slab row per sample
        const int o_hi = min(C2, (grp + 1) * MTG * 32);
        for (int o = grp * MTG * 32 + tid; o < o_hi; o += FU_THREADS) {
            float nn = 0.0f, mean = 0.0f, m2 = 0.0f;
            for (int nt = 0; nt < NTL; ++nt) {
                const float* st = Yre + (nt * C2 + o) * 3;
                const float cn = st[0], cm = st[1], cq = st[2];
                const float tot = nn + cn;
                const float delta = cm - mean;
                mean += delta * (cn / tot);
                m2 += cq + delta * delta * (nn * cn / tot);
                nn = tot;
            }
            reinterpret_cast<float4*>(a.slab)[(size_t)b * C2 + o] = make_float4(nn, mean, m2, 0.0f);
        }
#ifdef FFC_TRACE
        __syncthreads();
        FU_STAMP(5);
        if (tid == 0) g_fu_trace[8 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
#endif
        return;
    } else if (a.shuf) {
        // 4+5. lane y reads spectrum row bitrev(y), the inverse column DFTs run across the channel's H
        //      lanes (lane_ifft_dit, ortho scale folded in) and leave row y in lane y for its C2R
        for (int r = tid; r < C * H; r += FU_THREADS) {
            const int ch = r / H, y = r - ch * H;
            const int yo = lane_brev<H>(y);
            const float* yr = Yre + (ch * H + yo) * WP;
            const float* yi = Yim + (ch * H + yo) * WP;
            float xr[WP], xi[WP], re[W];
#pragma unroll
            for (int k = 0; k < WP; ++k) {
                xr[k] = yr[k];
                xi[k] = yi[k];
            }
            lane_ifft_dit<H, WP>(xr, xi, y, a.norm);
            irfft_reg<W>(xr, xi, re);
            if (a.residual) {
                float s[W];
                load_s_row<W, UP>(a, insc, b, ch, y, H, s);
#pragma unroll
                for (int x = 0; x < W; ++x) re[x] += s[x];
            }
            store_row<W>(a.out + ((size_t)(b * C + ch) * H + y) * W, re);
        }
    } else {
        // 4. inverse column C2C over H, ortho scale
        for (int q = tid; q < C * WP; q += FU_THREADS) {
            const int ch = q / WP, k = q - ch * WP;
            float* yr = Yre + ch * NB + k;
            float* yi = Yim + ch * NB + k;
            float re[H], im[H];
#pragma unroll
            for (int y = 0; y < H; ++y) {
                re[y] = yr[y * WP];
                im[y] = yi[y * WP];
            }
            fft_reg<H, true>(re, im);
#pragma unroll
            for (int y = 0; y < H; ++y) {
                yr[y * WP] = re[y] * a.norm;
                yi[y * WP] = im[y] * a.norm;
            }
        }
        __syncthreads();
        FU_STAMP(4);

        // 5. per-row C2R over W (imaginary part of bins 0 and W/2 ignored) + residual
        for (int r = tid; r < C * H; r += FU_THREADS) {
            const int ch = r / H, y = r - ch * H;
            const float* yr = Yre + (ch * H + y) * WP;
            const float* yi = Yim + (ch * H + y) * WP;
            float xr[WP], xi[WP], re[W];
#pragma unroll
            for (int k = 0; k < WP; ++k) {
                xr[k] = yr[k];
                xi[k] = yi[k];
            }
            irfft_reg<W>(xr, xi, re);   // W/2-point complex inverse FFT (fft_common.h)
            if (a.residual) {
                float s[W];
                load_s_row<W, UP>(a, insc, b, ch, y, H, s);
#pragma unroll
                for (int x = 0; x < W; ++x) re[x] += s[x];
            }
            store_row<W>(a.out + ((size_t)(b * C + ch) * H + y) * W, re);
        }
#ifdef FFC_TRACE
        __syncthreads();
        FU_STAMP(5);
        if (tid == 0) g_fu_trace[8 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
#endif
    }
}

// ---------------------------------------------------------------- pass 0 over bin groups
// fu_kernel's pass 0 holds a sample's whole spectrum (4 planes) in LDS: at ffc2 / ffc3 of the
// generator that is 133-146 KB, one workgroup per CU, and at B = 256 the grid is exactly one round
// of 256 workgroups whose load -> row R2C -> column FFT -> mix -> statistics phases run back to back
// with nothing to overlap them (VERDICT r05 "occupancy-capped").  Pass 0 needs no Y planes, and a
// column FFT needs only its own column: here G workgroups share a sample, workgroup g keeping only
// the half-spectrum columns k in [g KW0, g KW0 + kw) (KW0 = ceil((W/2+1) / G)).  Each repeats the
// row R2C (a few hundred VALU per row) but holds, transforms, mixes and spills only its columns:
// LDS Z (2 C H KW0 floats) + tile statistics + a 16-row statistics scratch, 2-4 workgroups per CU.
//   spill layout (per sample and channel o, still NB floats): [g][y][k - g KW0] -- workgroup g
//   stores whole 32-bin runs; pass 1 decodes it (fu_spill_bin).
//   slab rows: b G + g, each a partial over the workgroup's bins (the fold / reduce merge them).
// Grid: blockIdx = g B + b, so a sample's groups share an XCD (B % 8 == 0) and its t planes' second
// read comes from that XCD's L2.
// tile_row_stats (ffc_internal.h) in two rounds of 16 rows through a 16 x 33 per-wave scratch (half
// the LDS): lane quad 4 o' .. 4 o' + 3 reduces row 16 R + o' over 8 columns each (quad DPP sums,
// bit-identical in the quad).  mean[R], m2[R]: row 16 R + (lane >> 2), valid in every lane.
__device__ __forceinline__ void tile_row_stats16(const floatx16& acc, int nv, float* scratch, float (&mean)[2],
                                                 float (&m2)[2]) {
    const int lane = threadIdx.x & 63, h = lane >> 5, col = lane & 31;
    const int o = lane >> 2, c0 = (lane & 3) * 8;
#pragma unroll
    for (int R = 0; R < 2; ++R) {
        wave_lds_sync();   // the previous round's (or tile's) reads of the scratch precede these writes
#pragma unroll
        for (int r = 8 * R; r < 8 * R + 8; ++r) scratch[((r & 3) + 8 * ((r >> 2) & 1) + 4 * h) * 33 + col] = acc[r];
        wave_lds_sync();   // another lane's writes precede these reads (one wave: LDS in order)
        float v[8];
        float s = 0.0f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            v[j] = scratch[o * 33 + c0 + j];
            if (c0 + j < nv) s += v[j];
        }
        s += ffc::dpp_full<0xB1>(s);
        s += ffc::dpp_full<0x4E>(s);
        const float mu = s / (float)nv;
        float q = 0.0f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float d = v[j] - mu;
            if (c0 + j < nv) q = fmaf(d, d, q);
        }
        q += ffc::dpp_full<0xB1>(q);
        q += ffc::dpp_full<0x4E>(q);
        mean[R] = mu;
        m2[R] = q;
    }
    wave_lds_sync();
}

constexpr int FU_KG_SCRATCH = (FU_THREADS / 64) * 16 * 33;

// one bin group's body: group GI, columns K0 .. K0 + KW - 1 (compile-time strides and register
// indices: the column lines' LDS offsets become immediates)
template <int H, int W, int UP, int G, int GI>
__device__ __forceinline__ void fu_kg_body(const FuArgs& a, float* smem) {
    using K = FuKg<W, G>;
    constexpr int WP = K::WP, NB = H * WP, KW0 = K::KW0;
    constexpr int ZPL = H * KW0;                          // LDS bins of one channel (the widest group)
    constexpr int K0 = GI * KW0, KW = GI < G - 1 ? KW0 : K::KWL;
    constexpr int NBL = H * KW;                           // this group's bins per channel
    constexpr int NTL = (NBL + 31) / 32;
    const int C = a.C, C2 = 2 * C;
    const int b = blockIdx.x % a.B;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, col = lane & 31;
    float* Zre = smem;                                    // [C][H][KW] (channel stride NBL)
    float* Zim = Zre + C * ZPL;
    float* Wm = Zim + C * ZPL;                            // split mix weight (when staged: wm_lds)
    float* st = smem + a.scr_off;                         // tile statistics [NTL][C2][3]
    float* scr = st + ((ZPL + 31) / 32) * C2 * 3;         // per-wave 16 x 33 row scratch
    const float* insc = smem + a.bn_off;                  // folded input affine: scale [C] | shift [C]

    // 1. row R2C of every (channel, row) on a W/2-point complex FFT (rfft_reg); this group's columns
    FU_STAMP(1);
    for (int r = tid; r < C * H; r += FU_THREADS) {
        const int ch = r / H, y = r - ch * H;
        float sv[W], re[WP], im[WP];
        load_s_row<W, UP>(a, insc, b, ch, y, H, sv);
        rfft_reg<W>(sv, re, im);
        float* zr = Zre + ch * NBL + y * KW;
        float* zi = Zim + ch * NBL + y * KW;
#pragma unroll
        for (int kk = 0; kk < KW; ++kk) {
            zr[kk] = re[K0 + kk];
            zi[kk] = im[K0 + kk];
        }
    }
    // the mix weight's LDS-DMA (the kernel's first loads) is tracked by vmcnt only: this wave's
    // copies landed before the barrier, so every wave may read Wm after it
    if (a.wm_lds) ffc::dma_wait();
    __syncthreads();
    FU_STAMP(2);

    // 2. column C2C over H of this group's columns, ortho scale
    for (int q = tid; q < C * KW; q += FU_THREADS) {
        const int ch = q / KW, kk = q - ch * KW;
        float* zr = Zre + ch * NBL + kk;
        float* zi = Zim + ch * NBL + kk;
        float re[H], im[H];
#pragma unroll
        for (int y = 0; y < H; ++y) {
            re[y] = zr[y * KW];
            im[y] = zi[y * KW];
        }
        fft_reg<H, false>(re, im);
#pragma unroll
        for (int y = 0; y < H; ++y) {
            zr[y * KW] = re[y] * a.norm;
            zi[y * KW] = im[y] * a.norm;
        }
    }
    __syncthreads();
    FU_STAMP(3);

    // 3. mix (pre-split weight fragments, split-bf16 products) -> raw Y spill + tile statistics
    const int MT = (C2 + 31) >> 5, QN = C >> 3;
    float* ysb = a.yspill + (size_t)b * C2 * NB + GI * ZPL;
    for (int tile = wave; tile < MT * NTL; tile += FU_THREADS / 64) {
        const int mt = tile % MT, nt = tile / MT;
        floatx16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
        const float* zp = (h ? Zim : Zre) + nt * 32 + col;
        const uint16_t* w3 = (a.wm_lds ? reinterpret_cast<const uint16_t*>(Wm) : a.wmix3) +
                             (size_t)mt * QN * 1536 + lane * 8;
#pragma unroll 2
        for (int q = 0; q < QN; ++q) {
            Split3 av;
            av.hi = *reinterpret_cast<const bf16x8*>(w3 + q * 1536);
            av.mid = *reinterpret_cast<const bf16x8*>(w3 + q * 1536 + 512);
            av.lo = *reinterpret_cast<const bf16x8*>(w3 + q * 1536 + 1024);
            float zv[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) zv[j] = zp[(8 * q + j) * NBL];
            acc = mfma_split3(av, split3(zv), acc);
        }
        const int n = nt * 32 + col;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int o = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (n < NBL && o < C2) ysb[(size_t)o * NB + n] = acc[r];
        }
        const int nv = min(32, NBL - nt * 32);
        float mean[2], m2[2];
        tile_row_stats16(acc, nv, scr + wave * 16 * 33, mean, m2);
        if ((lane & 3) == 0) {
#pragma unroll
            for (int R = 0; R < 2; ++R) {
                const int o = mt * 32 + 16 * R + (lane >> 2);
                if (o < C2) {
                    float* s3 = st + (nt * C2 + o) * 3;
                    s3[0] = (float)nv;
                    s3[1] = mean[R];
                    s3[2] = m2[R];
                }
            }
        }
    }
    __syncthreads();
    FU_STAMP(4);
    // 4. the tiles' partials of each channel (Chan et al., tile order) -> slab row GI B + b
    for (int o = tid; o < C2; o += FU_THREADS) {
        float nn = 0.0f, mean = 0.0f, m2 = 0.0f;
        for (int nt = 0; nt < NTL; ++nt) {
            const float* s3 = st + (nt * C2 + o) * 3;
            const float cn = s3[0], cm = s3[1], cq = s3[2];
            const float tot = nn + cn;
            const float delta = cm - mean;
            mean += delta * (cn / tot);
            m2 += cq + delta * delta * (nn * cn / tot);
            nn = tot;
        }
        reinterpret_cast<float4*>(a.slab)[((size_t)GI * a.B + b) * C2 + o] = make_float4(nn, mean, m2, 0.0f);
    }
#ifdef FFC_TRACE
    __syncthreads();
    FU_STAMP(5);
    if (tid == 0) g_fu_trace[8 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
#endif
}

template <int H, int W, int UP, int G>
__global__ __launch_bounds__(FU_THREADS, 4) void fu_pass0_kg_kernel(FuArgs a) {   // 4 waves / SIMD: 2 WGs / CU
    static_assert(G == 2, "two bin groups");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int C = a.C, tid = threadIdx.x;
    const int g = blockIdx.x / a.B;
#ifdef FFC_TRACE
    if (tid == 0) g_fu_trace[8 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
#endif
    FU_STAMP(0);
    if (a.wm_lds) {
        typedef __attribute__((address_space(1))) void* gptr_t;
        typedef __attribute__((address_space(3))) void* lptr_t;
        float* Wm = smem + 2 * C * (H * FuKg<W, G>::KW0);
        const int n4 = (a.Mpad >> 5) * (C >> 3) * 192;   // 16-byte groups of the split pieces
        for (int i0 = 0; i0 < n4; i0 += FU_THREADS) {
            if (i0 + (tid & ~63) < n4) {
                const int i = min(i0 + tid, n4 - 1);
                __builtin_amdgcn_global_load_lds((gptr_t)(reinterpret_cast<const float*>(a.wmix3) + 4 * (size_t)i),
                                                 (lptr_t)(Wm + 4 * (i0 + (tid & ~63))), 16, 0, 0);
            }
        }
    }
    if (a.has_in_fold)
        ffc::bn_fold_block<FU_THREADS>(a.in_fold, smem + a.bn_off, smem + a.bn_off + C, blockIdx.x == 0,
                                       reinterpret_cast<double*>(smem));
    if (g == 0)
        fu_kg_body<H, W, UP, G, 0>(a, smem);
    else
        fu_kg_body<H, W, UP, G, 1>(a, smem);
}

// Pass 1 from the spilled Y, split over channel groups: one wave per (sample, 64 / H channels).
// fu_kernel's pass 1 runs a whole sample per 8-wave workgroup, one workgroup per CU at B = 256, so
// its load / column-IFFT / row-C2R phases cannot overlap; pass 1 needs no cross-channel data (the
// mix ran in pass 0), so here every wave takes 64 / H channels (64 rows, (64 / H) (W/2 + 1) column
// lines) and many waves share a CU.  Same arithmetic per line as fu_kernel (bit-identical).
template <int H, int W, int UP, int G>
__global__ __launch_bounds__(64) void fu_pass1_split_kernel(FuArgs a) {
    constexpr int WP = W / 2 + 1;
    constexpr int NB = H * WP;
    constexpr int CPG = 64 / H;   // channels per wave
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int C = a.C, C2 = 2 * C;
    const int ngroups = C / CPG;
    const int b = blockIdx.x / ngroups, c0 = (blockIdx.x - b * ngroups) * CPG;
    const int tid = threadIdx.x;
    float* Yre = smem;
    float* Yim = Yre + CPG * NB;
    __shared__ float fbn[2][2 * CPG];
    const float* bsc = a.bn_scale + 2 * c0;
    const float* bsh = a.bn_shift + 2 * c0;
    // this lane's residual row (s = transform(t) of row tid), loaded first: its latency sits under
    // the fold and the Y load instead of after the column IFFT
    float sres[W];
    if (a.residual) {
        load_s_row<W, UP>(a, nullptr, b, c0 + tid / H, tid % H, H, sres);
    } else {
#pragma unroll
        for (int x = 0; x < W; ++x) sres[x] = 0.0f;
    }
    if (a.has_mix_fold) {
        // the FU's BN of this wave's 2 CPG spectral channels, folded here: 64 / (2 CPG) lanes per
        // channel (ffc::bn_fold_channels), sample 0's waves lead
        constexpr int LPC = 64 / (2 * CPG);
        const int ol = tid / LPC;
        float fs, fh;
        ffc::bn_fold_channels<LPC>(a.mix_fold, 2 * c0 + ol, b == 0, fs, fh);
        if ((tid & (LPC - 1)) == 0) {
            fbn[0][ol] = fs;
            fbn[1][ol] = fh;
        }
        if (blockIdx.x == 0 && tid == 0 && a.mix_fold.update_running) *a.mix_fold.num_batches_tracked += 1;
        __syncthreads();
        bsc = fbn[0];
        bsh = fbn[1];
    }
    // Y rows 2 c0 .. 2 (c0 + CPG) of this sample -> BN + ReLU -> the Y planes
    const float4* ys = reinterpret_cast<const float4*>(a.yspill + ((size_t)b * C2 + 2 * c0) * NB);
    for (int i = tid; i < 2 * CPG * NB / 4; i += 64) {
        const int ol = (4 * i) / NB, n = 4 * i - ol * NB;
        const float4 v = ys[i];
        const float sc = bsc[ol], sh = bsh[ol];
        float* dst = ((ol & 1) ? Yim : Yre) + (ol >> 1) * NB;
        spill_to_plane<H, W, G>(dst, n, v, sc, sh);
    }
    __syncthreads();
    if (a.shuf) {   // lane (ch, y): row bitrev(y) in, inverse column DFTs across the H lanes, row y out
        const int ch = tid / H, y = tid - ch * H;
        const int yo = lane_brev<H>(y);
        const float* yr = Yre + (ch * H + yo) * WP;
        const float* yi = Yim + (ch * H + yo) * WP;
        float xr[WP], xi[WP], re[W];
#pragma unroll
        for (int k = 0; k < WP; ++k) {
            xr[k] = yr[k];
            xi[k] = yi[k];
        }
        lane_ifft_dit<H, WP>(xr, xi, y, a.norm);
        irfft_reg<W>(xr, xi, re);
#pragma unroll
        for (int x = 0; x < W; ++x) re[x] += sres[x];
        store_row<W>(a.out + ((size_t)(b * C + c0 + ch) * H + y) * W, re);
        return;
    }
    for (int q = tid; q < CPG * WP; q += 64) {   // inverse column C2C over H, ortho scale
        const int ch = q / WP, k = q - ch * WP;
        float* yr = Yre + ch * NB + k;
        float* yi = Yim + ch * NB + k;
        float re[H], im[H];
#pragma unroll
        for (int y = 0; y < H; ++y) {
            re[y] = yr[y * WP];
            im[y] = yi[y * WP];
        }
        fft_reg<H, true>(re, im);
#pragma unroll
        for (int y = 0; y < H; ++y) {
            yr[y * WP] = re[y] * a.norm;
            yi[y * WP] = im[y] * a.norm;
        }
    }
    __syncthreads();
    {   // per-row C2R over W + residual: one row per lane (CPG * H = 64)
        const int ch = tid / H, y = tid - ch * H;
        const float* yr = Yre + (ch * H + y) * WP;
        const float* yi = Yim + (ch * H + y) * WP;
        float xr[WP], xi[WP], re[W];
#pragma unroll
        for (int k = 0; k < WP; ++k) {
            xr[k] = yr[k];
            xi[k] = yi[k];
        }
        irfft_reg<W>(xr, xi, re);   // W/2-point complex inverse FFT (fft_common.h)
#pragma unroll
        for (int x = 0; x < W; ++x) re[x] += sres[x];
        store_row<W>(a.out + ((size_t)(b * C + c0 + ch) * H + y) * W, re);
    }
}

// out[k][o] = w[o][k] for o < R (zero for R <= o < Rpad); w is (R, K) row-major
__global__ void pack_transpose_kernel(const float* __restrict__ w, int R, int K, int Rpad, float* __restrict__ wt) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= K * Rpad) return;
    const int k = idx / Rpad, o = idx - k * Rpad;
    wt[idx] = (o < R) ? w[(size_t)o * K + k] : 0.0f;
}

typedef void (*FuKernel)(FuArgs);

template <int H, int W>
FuKernel pick_up_pass(int up, int pass) {
    if (up == 1) return pass == 0 ? fu_kernel<H, W, 1, 0> : fu_kernel<H, W, 1, 1>;
    return pass == 0 ? fu_kernel<H, W, 2, 0> : fu_kernel<H, W, 2, 1>;
}

template <int H>
FuKernel pick_w(int W, int up, int pass) {
    switch (W) {
        case 4: return pick_up_pass<H, 4>(up, pass);
        case 8: return pick_up_pass<H, 8>(up, pass);
        case 16: return pick_up_pass<H, 16>(up, pass);
        case 32: return pick_up_pass<H, 32>(up, pass);
    }
    return nullptr;
}

FuKernel pick_kernel(int H, int W, int up, int pass) {
    switch (H) {
        case 4: return pick_w<4>(W, up, pass);
        case 8: return pick_w<8>(W, up, pass);
        case 16: return pick_w<16>(W, up, pass);
        case 32: return pick_w<32>(W, up, pass);
    }
    return nullptr;
}

bool pow2_in(int v, int lo, int hi) { return v >= lo && v <= hi && (v & (v - 1)) == 0; }

template <int H, int W, int UP>
FuKernel pick_split_g(int kgroups) {
    return kgroups == 2 ? fu_pass1_split_kernel<H, W, UP, 2> : fu_pass1_split_kernel<H, W, UP, 1>;
}
FuKernel pick_split(int H, int W, int up, int kgroups) {
    if (H != W || !(kgroups == 1 || kgroups == 2)) return nullptr;
    switch (H) {
        case 8: return up == 1 ? pick_split_g<8, 8, 1>(kgroups) : pick_split_g<8, 8, 2>(kgroups);
        case 16: return up == 1 ? pick_split_g<16, 16, 1>(kgroups) : pick_split_g<16, 16, 2>(kgroups);
        case 32: return up == 1 ? pick_split_g<32, 32, 1>(kgroups) : pick_split_g<32, 32, 2>(kgroups);
    }
    return nullptr;
}
// pass 0 over G = 2 bin groups (fu_pass0_kg_kernel): square 8^2 .. 32^2 planes, pre-split weights
FuKernel pick_kg(int H, int W, int up) {
    if (H != W) return nullptr;
    switch (H) {
        case 8: return up == 1 ? fu_pass0_kg_kernel<8, 8, 1, 2> : fu_pass0_kg_kernel<8, 8, 2, 2>;
        case 16: return up == 1 ? fu_pass0_kg_kernel<16, 16, 1, 2> : fu_pass0_kg_kernel<16, 16, 2, 2>;
        case 32: return up == 1 ? fu_pass0_kg_kernel<32, 32, 1, 2> : fu_pass0_kg_kernel<32, 32, 2, 2>;
    }
    return nullptr;
}
// LDS of fu_pass0_kg_kernel: Z (2 C H KW0), the split weight when wm (staged), tile statistics
// (ceil(H KW0 / 32) x 2C x 3), the per-wave 16-row scratch, the folded input affine (2C)
struct KgLayout {
    size_t bytes;
    int wm_lds, scr_off, bn_off;
};
KgLayout kg_layout(int C, int H, int W, int G, bool wm) {
    const int WP = W / 2 + 1, KW0 = (WP + G - 1) / G, ZPL = H * KW0;
    const size_t z = (size_t)2 * C * ZPL;
    const size_t wfl = wm ? ((size_t)((2 * C + 31) / 32) * (C / 8) * 768 + 255) / 256 * 256 : 0;
    const size_t stf = (size_t)((ZPL + 31) / 32) * 2 * C * 3;
    const size_t floats = z + wfl + stf + FU_KG_SCRATCH + 2 * (size_t)C;
    return {4 * floats, wm ? 1 : 0, (int)(z + wfl), (int)(z + wfl + stf + FU_KG_SCRATCH)};
}
// FFC_FU_KGROUPS: 2 = on, anything else off (fu_kernel's pass 0, one workgroup or M-tile groups per sample)
int fu_kgroups_env() {
    static const int v = [] {
        const char* e = std::getenv("FFC_FU_KGROUPS");
        return e ? std::atoi(e) : -1;
    }();
    return v;
}

// FFC_FU_MFMA=split: the fused mix on the split-bf16 products instead of the exact f32-input MFMA.
// Off by default: measured neutral (gen64 B = 256 fu_pass0 51 vs 52 us per step, B = 32 the same,
// r05f) -- the fused mix waits on its LDS operand reads and the per-tile statistics, not the MFMA
bool fu_mix3_on() {
    static const bool on = [] {
        const char* e = std::getenv("FFC_FU_MFMA");
        return e && e[0] == 's';
    }();
    return on;
}
// with pre-split weights (ffc_fu_forward_ex3) the split mix is the default; FFC_FU_MFMA=f32 keeps the
// exact f32-input MFMA (A/B)
bool fu_mix_f32_forced() {
    static const bool on = [] {
        const char* e = std::getenv("FFC_FU_MFMA");
        return e && e[0] == 'f';
    }();
    return on;
}
// FFC_FU_SHUF=1: the column DFTs across lanes (fft_common.h lane_fft_dif / lane_ifft_dit) instead of
// through LDS (one lane per column line).  Off by default: measured level with the LDS column pass at
// gen64 B = 256 and B = 32 (round 6) -- the row / column phases are VALU-issue bound, and
// the lane form spends in butterfly arithmetic on every lane what it saves in LDS traffic and barriers
bool fu_shuf_on() {
    static const bool on = [] {
        const char* e = std::getenv("FFC_FU_SHUF");
        return e && e[0] == '1';
    }();
    return on;
}
// FFC_FU_SPLIT=0: pass 1 as one workgroup per sample (fu_kernel) for A/B runs
bool fu_split_on() {
    static const bool on = [] {
        const char* e = std::getenv("FFC_FU_SPLIT");
        return !(e && e[0] == '0');
    }();
    return on;
}

// LDS plan: Z/Y planes, then the mix weight when it fits, then the stats scratch unless it fits in
// the Y-imaginary plane.  bytes = 0: unsupported.
struct FuLayout {
    size_t bytes;
    int wm_lds, scr_off, bn_off;
};
// floats of the LDS weight region holding the split pieces: (Mpad / 32) x (C / 8) fragments of 3 KB
__host__ inline size_t fu_wm3_floats(int C) {
    const size_t Mpad = (size_t)(2 * C + 31) / 32 * 32;
    return ((Mpad / 32) * (size_t)(C / 8) * 768 + 255) / 256 * 256;
}
FuLayout fu_layout(int C, int H, int W, bool packed = false) {
    const size_t plane = (size_t)C * H * (W / 2 + 1);
    const bool in_y = plane >= (size_t)FU_SCRATCH;
    for (int wm = 1; wm >= 0; --wm) {
        const size_t wfl = wm ? (packed ? fu_wm3_floats(C) : fu_wm_floats(C)) : 0;
        const size_t scr = in_y ? 0 : FU_SCRATCH;
        const size_t floats = 4 * plane + wfl + scr + 6 * (size_t)C;
        if (4 * floats <= 160 * 1024)
            return {4 * floats, wm, (int)(in_y ? 3 * plane : 4 * plane + wfl), (int)(4 * plane + wfl + scr)};
    }
    return {0, 0, 0, 0};
}



}  // namespace

#ifdef FFC_TRACE
extern "C" int ffc_debug_fu_trace_read(void* dst, size_t bytes) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_fu_trace), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

extern "C" size_t ffc_fu_lds_bytes(int C, int H, int W) {
    if (C <= 0 || C > 4096 || !pow2_in(H, 4, 32) || !pow2_in(W, 4, 32)) return 0;   // C > 4096 never fits LDS
    return fu_layout(C, H, W).bytes;
}

extern "C" int ffc_fu_forward(const float* t, int B, int C, int H, int W, int up, const float* in_scale,
                              const float* in_shift, int in_relu, const float* wmixT, int pass,
                              float* stats_slab, const float* bn_scale, const float* bn_shift, int residual,
                              float* out, void* stream) {
    return ffc_fu_forward_ex(t, B, C, H, W, up, in_scale, in_shift, in_relu, wmixT, pass, stats_slab, bn_scale,
                             bn_shift, residual, out, nullptr, nullptr, nullptr, stream);
}

namespace {
__global__ void fu_pack_mix3_kernel(const float* __restrict__ wmixT, int C, int Mpad, uint16_t* __restrict__ out) {
    const int QN = C / 8, n = (Mpad / 32) * QN * 64;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int lane = i & 63, fr = i >> 6;   // fragment fr = M-tile * QN + k-block
        const int mt = fr / QN, q = fr - mt * QN;
        const int h = lane >> 5, col = lane & 31;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = wmixT[(size_t)(2 * (8 * q + j) + h) * Mpad + mt * 32 + col];
        const Split3 sp = split3(v);
        uint16_t* d = out + (size_t)fr * 1536 + lane * 8;
        *reinterpret_cast<u32x4*>(d) = __builtin_bit_cast(u32x4, sp.hi);
        *reinterpret_cast<u32x4*>(d + 512) = __builtin_bit_cast(u32x4, sp.mid);
        *reinterpret_cast<u32x4*>(d + 1024) = __builtin_bit_cast(u32x4, sp.lo);
    }
}
}  // namespace

extern "C" size_t ffc_fu_mix3_elems(int C) {
    if (C <= 0 || C % 8 != 0) return 0;
    return (size_t)((2 * C + 31) / 32) * (C / 8) * 1536;
}

extern "C" int ffc_fu_pack_mix3(const float* wmixT, int C, uint16_t* wmix3, void* stream) {
    FFC_CHECK_ARG(wmixT && wmix3 && C > 0 && C % 8 == 0, "ffc_fu_pack_mix3: bad args (C % 8 == 0)");
    FFC_CHECK_ARG((reinterpret_cast<uintptr_t>(wmix3) & 15) == 0, "ffc_fu_pack_mix3: wmix3 must be 16-byte aligned");
    const int Mpad = (2 * C + 31) / 32 * 32;
    const int n = (Mpad / 32) * (C / 8) * 64;
    hipLaunchKernelGGL(fu_pack_mix3_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, wmixT, C, Mpad,
                       wmix3);
    return ffc::launch_status("ffc_fu_pack_mix3");
}

static int fu_forward_impl(const float* t, int B, int C, int H, int W, int up, const float* in_scale,
                           const float* in_shift, int in_relu, const float* wmixT, const uint16_t* wmix3, int pass,
                           float* stats_slab, const float* bn_scale, const float* bn_shift, int residual, float* out,
                           const ffc_bn_fold* in_fold, const ffc_bn_fold* mix_fold, float* yspill, int kgroups,
                           void* stream);

// Off by default (FFC_FU_KGROUPS=2 turns it on): measured on MI355X (r06c / r06e, same-box A/B) the
// bin-group pass 0 is 0-1 us faster per layer at B = 256 and 64, and its doubled slab rows cost the
// per-channel fold of ffc3's mix BN at B = 256 (a finalize launch more): gen64 0.4286 -> 0.4309 ms.
extern "C" int ffc_fu_kgroups(int B, int C, int H, int W) {
    const int env = fu_kgroups_env();
    if (B <= 0 || C <= 0 || C % 8 != 0 || fu_mix_f32_forced() || env != 2 || H != W || !pick_kg(H, W, 1)) return 1;
    if (kg_layout(C, H, W, 2, false).bytes > 80 * 1024) return 1;   // two workgroups per CU or not at all
    return 2;
}

extern "C" int ffc_fu_slab_rows(int B, int C, int H, int W, int kgroups) {
    if (B <= 0 || C <= 0 || H <= 0 || W <= 0) return 0;
    return B * (kgroups == 2 ? 2 : 1);
}

extern "C" int ffc_fu_forward_ex(const float* t, int B, int C, int H, int W, int up, const float* in_scale,
                                 const float* in_shift, int in_relu, const float* wmixT, int pass, float* stats_slab,
                                 const float* bn_scale, const float* bn_shift, int residual, float* out,
                                 const ffc_bn_fold* in_fold, const ffc_bn_fold* mix_fold, float* yspill,
                                 void* stream) {
    return fu_forward_impl(t, B, C, H, W, up, in_scale, in_shift, in_relu, wmixT, nullptr, pass, stats_slab, bn_scale,
                           bn_shift, residual, out, in_fold, mix_fold, yspill, 1, stream);
}

extern "C" int ffc_fu_forward_ex3(const float* t, int B, int C, int H, int W, int up, const float* in_scale,
                                  const float* in_shift, int in_relu, const float* wmixT, const uint16_t* wmix3,
                                  int pass, float* stats_slab, const float* bn_scale, const float* bn_shift,
                                  int residual, float* out, const ffc_bn_fold* in_fold, const ffc_bn_fold* mix_fold,
                                  float* yspill, void* stream) {
    FFC_CHECK_ARG(!wmix3 || (C % 8 == 0 && (reinterpret_cast<uintptr_t>(wmix3) & 15) == 0),
                  "ffc_fu_forward_ex3: wmix3 needs C % 8 == 0 and 16-byte alignment");
    return fu_forward_impl(t, B, C, H, W, up, in_scale, in_shift, in_relu, wmixT, wmix3, pass, stats_slab, bn_scale,
                           bn_shift, residual, out, in_fold, mix_fold, yspill, 1, stream);
}

extern "C" int ffc_fu_forward_ex4(const float* t, int B, int C, int H, int W, int up, const float* in_scale,
                                  const float* in_shift, int in_relu, const float* wmixT, const uint16_t* wmix3,
                                  int pass, float* stats_slab, const float* bn_scale, const float* bn_shift,
                                  int residual, float* out, const ffc_bn_fold* in_fold, const ffc_bn_fold* mix_fold,
                                  float* yspill, int kgroups, void* stream) {
    FFC_CHECK_ARG(kgroups == 1 || kgroups == 2, "ffc_fu_forward_ex4: kgroups must be 1 or 2");
    FFC_CHECK_ARG(kgroups == 1 || ffc_fu_kgroups(B, C, H, W) == 2,
                  "ffc_fu_forward_ex4: kgroups = 2 unsupported here (ffc_fu_kgroups)");
    FFC_CHECK_ARG(kgroups == 1 || (wmix3 && (reinterpret_cast<uintptr_t>(wmix3) & 15) == 0),
                  "ffc_fu_forward_ex4: kgroups = 2 needs the pre-split weight wmix3 (16-byte aligned)");
    FFC_CHECK_ARG(kgroups == 1 || pass == 1 || yspill, "ffc_fu_forward_ex4: kgroups = 2 pass 0 needs yspill");
    FFC_CHECK_ARG(!wmix3 || (C % 8 == 0 && (reinterpret_cast<uintptr_t>(wmix3) & 15) == 0),
                  "ffc_fu_forward_ex4: wmix3 needs C % 8 == 0 and 16-byte alignment");
    return fu_forward_impl(t, B, C, H, W, up, in_scale, in_shift, in_relu, wmixT, wmix3, pass, stats_slab, bn_scale,
                           bn_shift, residual, out, in_fold, mix_fold, yspill, kgroups, stream);
}

static int fu_forward_impl(const float* t, int B, int C, int H, int W, int up, const float* in_scale,
                           const float* in_shift, int in_relu, const float* wmixT, const uint16_t* wmix3, int pass,
                           float* stats_slab, const float* bn_scale, const float* bn_shift, int residual, float* out,
                           const ffc_bn_fold* in_fold, const ffc_bn_fold* mix_fold, float* yspill, int kgroups,
                           void* stream) {
    FFC_CHECK_ARG(B > 0 && C > 0, "ffc_fu_forward: B and C must be positive");
    FFC_CHECK_ARG(up == 1 || up == 2, "ffc_fu_forward: up must be 1 or 2");
    FFC_CHECK_ARG(pass == 0 || pass == 1, "ffc_fu_forward: pass must be 0 or 1");
    if (fu_mix_f32_forced() || C % 8 != 0) wmix3 = nullptr;
    const bool packed = wmix3 != nullptr;
    const size_t lds = ffc_fu_lds_bytes(C, H, W) > 0 ? fu_layout(C, H, W, packed).bytes : 0;
    FFC_CHECK_ARG(lds > 0, "ffc_fu_forward: unsupported (C,H,W): H,W must be powers of two in [4,32] "
                           "and 16*C*H*(W/2+1) <= 160 KiB");
    FFC_CHECK_ARG(t && wmixT, "ffc_fu_forward: null input");
    FFC_CHECK_ARG((in_scale == nullptr) == (in_shift == nullptr), "ffc_fu_forward: in_scale/in_shift pairing");
    if (pass == 0) FFC_CHECK_ARG(stats_slab != nullptr, "ffc_fu_forward: pass 0 needs stats_slab");
    if (pass == 1)
        FFC_CHECK_ARG(((bn_scale && bn_shift) || mix_fold) && out, "ffc_fu_forward: pass 1 needs bn_scale/shift/out");
    FFC_CHECK_ARG(!in_fold || (pass == 0 && !in_scale && in_fold->scale_out && in_fold->shift_out),
                  "ffc_fu_forward: in_fold is pass 0 only, replaces in_scale/in_shift and needs scale_out/shift_out");
    FFC_CHECK_ARG(!mix_fold || pass == 1, "ffc_fu_forward: mix_fold is pass 1 only");
    for (const ffc_bn_fold* f : {in_fold, mix_fold})
        FFC_CHECK_ARG(!f || ((f->moments || (f->slab && f->nrows > 0)) &&
                             (!f->update_running || (f->running_mean && f->running_var && f->num_batches_tracked))),
                      "ffc_fu_forward: incomplete ffc_bn_fold");
    FFC_CHECK_ARG(!in_fold || in_fold->C == C, "ffc_fu_forward: in_fold->C != C");
    FFC_CHECK_ARG(!mix_fold || mix_fold->C == 2 * C, "ffc_fu_forward: mix_fold->C != 2C");
    FFC_CHECK_ARG(((!in_fold || in_fold->moments) && (!mix_fold || mix_fold->moments)) ||
                      (size_t)16 * C * H * (W / 2 + 1) >= sizeof(double) * ffc::bn_fold_scratch_doubles(FU_THREADS),
                  "ffc_fu_forward: plane too small for an in-kernel BN fold (use bn_scale / in_scale)");
    FuKernel k = pick_kernel(H, W, up, pass);
    FFC_CHECK_ARG(k != nullptr, "ffc_fu_forward: no kernel instance");
    FuArgs a;
    a.t = t;
    a.in_scale = in_scale;
    a.in_shift = in_shift;
    a.has_in_affine = in_scale != nullptr;
    a.in_relu = in_relu;
    a.wmixT = wmixT;
    a.slab = stats_slab;
    a.bn_scale = bn_scale;
    a.bn_shift = bn_shift;
    a.out = out;
    a.C = C;
    a.Mpad = (2 * C + 31) / 32 * 32;
    a.residual = residual;
    a.norm = (float)(1.0 / std::sqrt((double)H * (double)W));
    const FuLayout lay = fu_layout(C, H, W, packed);
    a.wm_lds = lay.wm_lds;
    a.wmix3 = wmix3;
    a.w3_lds = packed && lay.wm_lds;
    a.scr_off = lay.scr_off;
    a.bn_off = lay.bn_off;
    a.has_in_fold = in_fold != nullptr;
    a.has_mix_fold = mix_fold != nullptr;
    if (in_fold) {
        a.in_fold = *in_fold;
        a.has_in_affine = 1;
    }
    if (mix_fold) a.mix_fold = *mix_fold;
    a.yspill = yspill;
    a.mix3 = (packed || fu_mix3_on()) && !fu_mix_f32_forced() && C % 8 == 0;
    // pass 0 of small batches over two workgroups per sample (M-tile groups) while the grid stays
    // within one workgroup per CU; FFC_FU_MGROUPS = 1 keeps one per sample, = 4 four (A/B)
    a.mgroups = 1;
    a.B = B;
    a.kgroups = kgroups;
    a.shuf = fu_shuf_on() && H >= 2 && H <= 32 ? 1 : 0;
    if (pass == 0 && kgroups == 2) {
        // pass 0 over two bin groups per sample (fu_pass0_kg_kernel): the split weight staged in LDS
        // while two workgroups still fit a CU, else read from L2
        FFC_CHECK_ARG(packed && yspill, "ffc_fu_forward: kgroups = 2 needs wmix3 and yspill");
        KgLayout kl = kg_layout(C, H, W, 2, true);
        if (kl.bytes > 80 * 1024) kl = kg_layout(C, H, W, 2, false);
        FFC_CHECK_ARG(kl.bytes <= 80 * 1024, "ffc_fu_forward: kgroups = 2 layout exceeds 80 KiB");
        FFC_CHECK_ARG(!in_fold || in_fold->moments || (size_t)kl.scr_off * 4 >= sizeof(double) * ffc::bn_fold_scratch_doubles(FU_THREADS),
                      "ffc_fu_forward: bin-group planes too small for the in-kernel bn1 fold");
        FuKernel kk = pick_kg(H, W, up);
        FFC_CHECK_ARG(kk != nullptr, "ffc_fu_forward: no bin-group kernel instance");
        a.wm_lds = kl.wm_lds;
        a.w3_lds = kl.wm_lds;
        a.scr_off = kl.scr_off;
        a.bn_off = kl.bn_off;
        if (kl.bytes > 64 * 1024) {
            static std::mutex mu;
            static std::set<const void*> raised;
            std::lock_guard<std::mutex> g(mu);
            if (!raised.count(reinterpret_cast<const void*>(kk))) {
                hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kk),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
                if (e != hipSuccess) {
                    ffc::set_error(std::string("ffc_fu_forward: hipFuncSetAttribute: ") + hipGetErrorString(e));
                    return FFC_E_LAUNCH;
                }
                raised.insert(reinterpret_cast<const void*>(kk));
            }
        }
        hipLaunchKernelGGL(kk, dim3((unsigned)B * 2), dim3(FU_THREADS), kl.bytes, (hipStream_t)stream, a);
        return ffc::launch_status("ffc_fu_forward");
    }
    if (pass == 0) {
        static const int force = [] {
            const char* e = std::getenv("FFC_FU_MGROUPS");
            return e ? std::atoi(e) : 0;
        }();
        const int MT = (2 * C + 31) / 32;
        int cus = 256, dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 256;
        for (int g : {4, 2}) {   // 2 unless forced: 4 groups repeat the FFTs once too often (B = 32: r05an)
            if (force <= 0 && g == 4) continue;
            if (force > 0 ? g == force : (long long)B * g <= cus) {
                if (MT % g == 0) {
                    a.mgroups = g;
                    break;
                }
            }
        }
    }
    if (lds > 64 * 1024) {
        // opt each instance into the full 160 KiB once (not a stream op; safe under capture)
        static std::mutex mu;
        static std::set<const void*> raised;
        std::lock_guard<std::mutex> g(mu);
        if (!raised.count(reinterpret_cast<const void*>(k))) {
            hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            if (e != hipSuccess) {
                ffc::set_error(std::string("ffc_fu_forward: hipFuncSetAttribute: ") + hipGetErrorString(e));
                return FFC_E_LAUNCH;
            }
            raised.insert(reinterpret_cast<const void*>(k));
        }
    }
    // pass 1 from the spill with the BN scale / shift given, or a mix fold the waves can take channel by
    // channel (momentum >= 0: ffc::bn_fold_channels): one wave per (sample, 64 / H channels)
    const bool chan_fold = mix_fold && mix_fold->momentum >= 0.0f && (2 * 64 / H) <= 64;
    if (pass == 1 && yspill && (!mix_fold || chan_fold) && fu_split_on() && H * W <= 64 * 64 && H <= 64 &&
        C % (64 / H) == 0) {
        FuKernel ks = pick_split(H, W, up, kgroups);
        if (ks) {
            const size_t slds = (size_t)2 * (64 / H) * H * (W / 2 + 1) * sizeof(float);
            hipLaunchKernelGGL(ks, dim3((unsigned)B * (C / (64 / H))), dim3(64), slds, (hipStream_t)stream, a);
            return ffc::launch_status("ffc_fu_forward");
        }
    }
    hipLaunchKernelGGL(k, dim3((unsigned)B * a.mgroups), dim3(FU_THREADS), lds, (hipStream_t)stream, a);
    return ffc::launch_status("ffc_fu_forward");
}

extern "C" int ffc_pack_transpose(const float* w, int R, int K, float* wT, void* stream) {
    FFC_CHECK_ARG(w && wT && R > 0 && K > 0, "ffc_pack_transpose: bad args");
    const int Rpad = (R + 31) / 32 * 32;
    const int n = K * Rpad;
    hipLaunchKernelGGL(pack_transpose_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, w, R, K,
                       Rpad, wT);
    return ffc::launch_status("ffc_pack_transpose");
}

extern "C" int ffc_fu_pack_mix(const float* w, int C2, float* wmixT, void* stream) {
    return ffc_pack_transpose(w, C2, C2, wmixT, stream);
}
