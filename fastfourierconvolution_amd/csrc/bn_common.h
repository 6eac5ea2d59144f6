// BatchNorm finalized inside the kernel that consumes it (ffc_bn_fold, include/ffc_amd.h): every
// workgroup merges the producer's {n, mean, M2} partial rows itself -- a fixed-order fp64 merge, so
// every workgroup forms bit-identical scale / shift -- and workgroup 0 alone updates the running
// statistics (nn.BatchNorm2d semantics, torch/nn/modules/batchnorm.py as called from
// layers/ffc/*.py) and writes the folded scale / shift out for later kernels.  Saves the separate
// reduce + finalize launch per BN (bn_se_kernels.hip) on the single-rank path.
#pragma once

#include "ffc_internal.h"

namespace ffc {

__device__ __forceinline__ double shfl_xor_f64(double v, int m) { return __shfl_xor(v, m, 64); }

// BLOCK threads (whole waves).  A wave reads 4 partial rows x 16 consecutive channels per load
// (four 256-byte segments); lane = 16 rg + oc.  The waves of a 16-channel block split its rows
// ((wave-in-block, rg) interleaved), merge rg with a fixed xor tree, and the wave partials meet
// in `scratch` (3 doubles per (block, wave, channel)) in wave order: a fixed merge order, so every
// workgroup forms bit-identical scale / shift.  Writes sc[o], sh[o] (LDS) for o < f.C; workgroup
// 0 (leader) also updates the running statistics, bumps num_batches_tracked (after every channel
// read it) and stores scale_out / shift_out.  Ends with a barrier.  scratch: bn_fold_scratch().
__host__ __device__ constexpr int bn_fold_scratch_doubles(int block) { return 3 * block / 4; }

// finalize of channel o from its raw moments {N, S = sum x, Q = sum x^2} (fp64): nn.BatchNorm2d's
// biased variance for the normalisation, unbiased over N * count_mult for running_var
__device__ __forceinline__ void bn_fold_finalize(const ffc_bn_fold& f, int o, double N, double S, double Q,
                                                 bool leader, int64_t nbt, float& scale, float& shift) {
    const double mu = S / N;
    double v = Q / N - mu * mu;
    if (v < 0.0) v = 0.0;
    const float mean = (float)mu, var = (float)v;
    const float inv = 1.0f / sqrtf(var + f.eps);
    const float g = f.gamma ? f.gamma[o] : 1.0f;
    const float b = f.beta ? f.beta[o] : 0.0f;
    scale = g * inv;
    shift = fmaf(-mean, scale, b);   // as bn_se_kernels.hip finalize_channel
    if (leader) {
        if (f.update_running) {
            float fm = f.momentum;
            if (fm < 0.0f) fm = 1.0f / (float)(nbt + 1);   // momentum=None: cumulative average
            const double nfull = N * (double)f.count_mult;
            const double unb = nfull > 1.0 ? v * nfull / (nfull - 1.0) : v;
            f.running_mean[o] = fmaf(fm, mean, (1.0f - fm) * f.running_mean[o]);
            f.running_var[o] = fmaf(fm, (float)unb, (1.0f - fm) * f.running_var[o]);
        }
        if (f.scale_out) f.scale_out[o] = scale;
        if (f.shift_out) f.shift_out[o] = shift;
    }
}

template <bool SWAP16>
__device__ __forceinline__ double permlane_sum_f64(double v);

template <int BLOCK>
__device__ void bn_fold_block(const ffc_bn_fold& f, float* sc, float* sh, bool leader, double* scratch) {
    constexpr int NW = BLOCK / 64;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (f.moments) {
        // SyncBN: the slab was reduced and all-reduced across ranks already (distributed.py); each
        // channel's finalize reads its three moments
        const int64_t nbt0 = (leader && f.update_running && f.momentum < 0.0f) ? *f.num_batches_tracked : 0;
        for (int o = tid; o < f.C; o += BLOCK) {
            float scale, shift;
            bn_fold_finalize(f, o, f.moments[3 * o], f.moments[3 * o + 1], f.moments[3 * o + 2], leader, nbt0, scale,
                             shift);
            sc[o] = scale;
            sh[o] = shift;
        }
        __syncthreads();   // every channel read num_batches_tracked before the bump
        if (leader && f.update_running && tid == 0) *f.num_batches_tracked += 1;
        return;
    }
    const int oc = lane & 15, rg = lane >> 4;
    const int nb = (f.C + 15) >> 4;                 // 16-channel blocks
    const int wpb = nb >= NW ? 1 : NW / nb;         // waves per block
    const int RS = 4 * wpb;                         // row stride of one lane
    const float4* slab = reinterpret_cast<const float4*>(f.slab);
    const int64_t nbt = (leader && f.update_running && f.momentum < 0.0f) ? *f.num_batches_tracked : 0;
    for (int cb0 = 0; cb0 < nb; cb0 += NW / wpb) {
        const int cb = cb0 + wave / wpb, k = wave % wpb;
        const int o = cb * 16 + oc;
        const bool live = cb < nb && wave < (NW / wpb) * wpb;
        const int oo = o < f.C ? o : f.C - 1;
        double n = 0.0, s = 0.0, q = 0.0;
        if (live) {
            int r = k * 4 + rg;
            for (; r + 3 * RS < f.nrows; r += 4 * RS) {   // four rows in flight per lane
                float4 e[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) e[u] = slab[(size_t)(r + u * RS) * f.C + oo];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const double en = e[u].x, em = e[u].y;
                    n += en;
                    s += en * em;
                    q += (double)e[u].z + en * em * em;
                }
            }
            for (; r < f.nrows; r += RS) {
                const float4 e = slab[(size_t)r * f.C + oo];
                const double en = e.x, em = e.y;
                n += en;
                s += en * em;
                q += (double)e.z + en * em * em;
            }
        }
        // v + v(lane ^ 16), then ^ 32: v_permlane16/32_swap, the same sums as a __shfl_xor pair
        n = permlane_sum_f64<true>(n);
        s = permlane_sum_f64<true>(s);
        q = permlane_sum_f64<true>(q);
        n = permlane_sum_f64<false>(n);
        s = permlane_sum_f64<false>(s);
        q = permlane_sum_f64<false>(q);
        if (live && rg == 0) {
            double* d = scratch + 3 * (wave * 16 + oc);
            d[0] = n;
            d[1] = s;
            d[2] = q;
        }
        __syncthreads();
        // one thread per channel of this round: the wpb wave partials in wave order, then finalize
        if (tid < (NW / wpb) * 16) {
            const int cbl = tid >> 4, c2 = cb0 + cbl, oc2 = tid & 15, o2 = c2 * 16 + oc2;
            if (c2 < nb && o2 < f.C) {
                double N = 0.0, S = 0.0, Q = 0.0;
                for (int w = 0; w < wpb; ++w) {
                    const double* d = scratch + 3 * ((cbl * wpb + w) * 16 + oc2);
                    N += d[0];
                    S += d[1];
                    Q += d[2];
                }
                float scale, shift;
                bn_fold_finalize(f, o2, N, S, Q, leader, nbt, scale, shift);
                sc[o2] = scale;
                sh[o2] = shift;
            }
        }
        __syncthreads();
    }
    if (leader && f.update_running && tid == 0) *f.num_batches_tracked += 1;
}

// Groups of L lanes (L a power of two <= 64) finalize one channel each -- channel o, given per lane --
// from that channel's partial rows only: for the consumers whose workgroups need one or a few
// channels (the staged Fourier unit's per-plane r2c / c2r: L = 64; the fused FU's per-wave pass 1:
// 64 / (2 x its channels)).  Rows (lane % L), + L, ... are merged per lane in that order (four loads
// in flight), then an xor tree over the group whose every level adds commutative pairs: the L lanes
// end with bit-identical totals, and so does every workgroup that folds channel o with the same L.
// Same finalize arithmetic as bn_fold_block.  leader: the running-statistics update and scale_out /
// shift_out of channel o (exactly one workgroup per channel leads); num_batches_tracked is bumped by
// the caller (one lane of the workgroup leading channel 0).  Needs momentum >= 0 (no read of
// num_batches_tracked: with per-channel leaders that read would race with the bump).
template <int CTRL>
__device__ __forceinline__ double dpp_full_f64(double v) {
    const long long iv = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)iv, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(iv >> 32), CTRL, 0xF, 0xF, false);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
// v + v of the lane 16 (SWAP16) or 32 lanes away, through v_permlane16_swap / v_permlane32_swap
template <bool SWAP16>
__device__ __forceinline__ double permlane_sum_f64(double v) {
    const long long iv = __builtin_bit_cast(long long, v);
    const int lo = (int)iv, hi = (int)(iv >> 32);
    const auto sl = SWAP16 ? __builtin_amdgcn_permlane16_swap(lo, lo, false, false)
                           : __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto sh = SWAP16 ? __builtin_amdgcn_permlane16_swap(hi, hi, false, false)
                           : __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    const double a = __builtin_bit_cast(double, ((long long)(int)sh[0] << 32) | (unsigned)(int)sl[0]);
    const double b = __builtin_bit_cast(double, ((long long)(int)sh[1] << 32) | (unsigned)(int)sl[1]);
    return a + b;
}
// sum over aligned groups of L lanes (L = 1 .. 64, a power of two) by symmetric DPP / permlane steps
// (each v += partner(v) with an involutive partner): every lane of a group holds the bit-identical sum
template <int L>
__device__ __forceinline__ double group_sum_f64(double v) {
#ifdef FFC_FOLD_SHFL
    for (int m = 1; m < L; m <<= 1) v += shfl_xor_f64(v, m);
    return v;
#endif
    if constexpr (L >= 2) v += dpp_full_f64<0xB1>(v);     // quad_perm [1,0,3,2]: lane ^ 1
    if constexpr (L >= 4) v += dpp_full_f64<0x4E>(v);     // quad_perm [2,3,0,1]: lane ^ 2
    if constexpr (L >= 8) v += dpp_full_f64<0x141>(v);    // row_half_mirror: the other quad of the 8
    if constexpr (L >= 16) v += dpp_full_f64<0x140>(v);   // row_mirror: the other 8 of the row
    if constexpr (L >= 32) v = permlane_sum_f64<true>(v);
    if constexpr (L >= 64) v = permlane_sum_f64<false>(v);
    return v;
}

template <int L>
__device__ inline void bn_fold_channels(const ffc_bn_fold& f, int o, bool leader, float& scale, float& shift) {
    static_assert(L >= 1 && L <= 64 && (L & (L - 1)) == 0, "lanes per channel");
    const int gl = threadIdx.x & (L - 1);
    // rows through a buffer descriptor: a row past the slab is a load at offset OOB that reads a
    // zero-count entry (a predicated load would compile to a branch and a wait per row)
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(f.slab, (unsigned long long)f.nrows * f.C * 16);
    double n = 0.0, s = 0.0, q = 0.0;
    if (f.moments) {   // SyncBN: moments reduced and all-reduced already; every lane reads them
        bn_fold_finalize(f, o, f.moments[3 * o], f.moments[3 * o + 1], f.moments[3 * o + 2], leader && gl == 0, 0,
                         scale, shift);
        return;
    }
    // up to 8 rows per lane in flight per round: one memory round trip for <= 8 L rows (the usual case)
    for (int r0 = gl; r0 < f.nrows; r0 += 8 * L) {
        floatx4 e[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int r = r0 + L * u;
#ifdef FFC_FOLD_PLAIN_LOADS   // DESIGN 10c probe: plain global loads instead of the buffer descriptor
            const float4 pv = r < f.nrows ? reinterpret_cast<const float4*>(f.slab)[(size_t)r * f.C + o]
                                          : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            e[u] = floatx4{pv.x, pv.y, pv.z, pv.w};
#else
            e[u] = buf_ld4(rs, r < f.nrows ? (unsigned)((r * f.C + o) * 16) : OOB);
#endif
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const double en = e[u][0], em = e[u][1];
            n += en;
            s += en * em;
            q += (double)e[u][2] + en * em * em;
        }
    }
    n = group_sum_f64<L>(n);
    s = group_sum_f64<L>(s);
    q = group_sum_f64<L>(q);
#ifdef FFC_FOLD_FIN1   // DESIGN 10c probe: the fp64 finalize in lane 0 of each group only (others: 0)
    scale = shift = 0.0f;
    if (gl == 0)
#endif
    bn_fold_finalize(f, o, n, s, q, leader && gl == 0, 0, scale, shift);   // momentum >= 0: nbt unused
}

// one whole wave per channel
__device__ inline void bn_fold_channel(const ffc_bn_fold& f, int o, bool leader, float& scale, float& shift) {
    bn_fold_channels<64>(f, o, leader, scale, shift);
}

}  // namespace ffc
