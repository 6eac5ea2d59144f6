// Fused SpectralTransform prologue for gfx950: one workgroup per sample.
//
// Replaces, for one sample at a time (layers/ffc/spectral_transform.py:79-89):
//   downsample (AvgPool2d(2) when pool=1; the x2 nearest Upsample commutes with everything
//   here and is applied later inside the Fourier-unit loads)
//   SELayer: gate = sigmoid(W2 relu(W1 mean_hw(x)))              (:12-28, hidden may be 0)
//   conv1 (1x1, no bias) on gate * x  ->  t                      (:52-53, :89)
//   per-sample BatchNorm partials {n, mean, M2} of t             (bn1, :57, :89)
// The sample (Cin x h x w) lives in LDS, conv1's pre-transposed weight streams from L2; conv1 runs on
// v_mfma_f32_32x32x2_f32 with the gate folded into the B-fragment read.
#include "ffc_internal.h"

#include <mutex>
#include <set>
#include <string>

namespace {

struct StArgs {
    const float* x;      // (B, Cin, H, W): H, W are the pre-pool dims when pool=1
    const float* w1;     // se fc.0 (hid, Cin)
    const float* w2;     // se fc.2 (Cin, hid)
    const float* wcT;    // conv1 weight transposed + zero padded: (Cin, Mpad), Mpad = ceil32(c)
    float* t;            // (B, c, h, w)
    float* slab;         // [B][c] float4
    float* gate_out;     // optional (B, Cin) copy of the gate (tests / debugging), may be null
    int Cin, H, W, pool, hid, c;
    const uint16_t* wc3; // optional: conv1 weight as split-bf16 MFMA fragments (ffc_st_pack_a3); else the
                         // exact f32-input MFMA on wcT
    int x_dma;           // sample copied by LDS-DMA (no pooling, 16-byte aligned rows)
    int split;           // workgroups per sample: each takes 1/split of conv1's output tiles
    // LDS layout (float offsets; -1: not staged, read from global)
    int gate_off, hv_off, st_off, red_off, scr_off, wt_off, w1_off, w2_off;
};

// 8 waves: at the batch sizes of a strong-scaling shard (32..256 samples = workgroups, at most one
// per CU) the kernel is latency-bound, and more waves shorten every phase (SE loops, conv1 split-K)
constexpr int ST_THREADS = 512;
constexpr int ST_WAVES = ST_THREADS / 64;

#ifdef FFC_TRACE
// Diagnostic build only: per workgroup {realtime start, end, s_memtime at phase boundaries 0..5}.
__device__ unsigned long long g_st_trace[8 * 4096];
#define ST_STAMP(i)                                                                         \
    do {                                                                                    \
        unsigned long long t_;                                                              \
        __builtin_amdgcn_sched_barrier(0);                                                  \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");         \
        __builtin_amdgcn_sched_barrier(0);                                                  \
        if (threadIdx.x == 0) g_st_trace[8 * blockIdx.x + 2 + (i)] = t_;                   \
    } while (0)
#else
#define ST_STAMP(i) do { } while (0)
#endif

__global__ __launch_bounds__(ST_THREADS) void st_prologue_kernel(StArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int b = blockIdx.x / a.split, sp = blockIdx.x % a.split;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int Cin = a.Cin, c = a.c;
    const int h = a.pool ? a.H / 2 : a.H, w = a.pool ? a.W / 2 : a.W;
    const int hw = h * w;
    const int Mpad = (c + 31) & ~31;
    float* xs = sm;                      // [Cin][hw]
    float* gate = sm + a.gate_off;       // [Cin]
    float* hv = sm + a.hv_off;           // [hid]
    float* st = sm + a.st_off;           // [ntile][c][3]
    float* red = sm + a.red_off;         // [ST_WAVES][16][64] split-K partials
    float* scr = sm + a.scr_off;         // [ST_WAVES][32 x 33] tile-stats scratch
    float* wt = sm + a.wt_off;           // [Cin][Mpad] conv1 weight (when staged)
    const int hid = a.hid;

#ifdef FFC_TRACE
    if (tid == 0) g_st_trace[8 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
#endif
    ST_STAMP(0);
    // 1. sample, conv1 weight and SE weights -> LDS, all in flight at once (LDS-DMA; the 2x2
    //    average pool, when present, on the way in through registers)
    const float* xb = a.x + (size_t)b * Cin * a.H * a.W;
    if (a.wt_off >= 0) ffc::dma_copy16(a.wcT, wt, Cin * Mpad / 4, tid, ST_THREADS);
    if (a.w1_off >= 0) {
        ffc::dma_copy16(a.w1, sm + a.w1_off, hid * Cin / 4, tid, ST_THREADS);
        ffc::dma_copy16(a.w2, sm + a.w2_off, Cin * hid / 4, tid, ST_THREADS);
    }
    if (!a.pool) {
        const int n = Cin * hw;
        if (a.x_dma) {
            ffc::dma_copy16(xb, xs, n / 4, tid, ST_THREADS);
        } else {
            for (int i = tid; i < n; i += ST_THREADS) xs[i] = xb[i];
        }
    } else {
        for (int i = tid; i < Cin * hw; i += ST_THREADS) {
            const int ch = i / hw, r = i - ch * hw, yy = r / w, xx = r - yy * w;
            const float* q = xb + ((size_t)ch * a.H + 2 * yy) * a.W + 2 * xx;
            xs[i] = (((q[0] + q[1]) + q[a.W]) + q[a.W + 1]) * 0.25f;
        }
    }
    ffc::dma_wait();
    __syncthreads();
    ST_STAMP(1);

    // 2. SE gate.  Reductions run over 16-lane DPP rows (no shuffle chains): row q of the
    //    block (16 lanes, consecutive pixels / inputs: conflict-free LDS) owns one channel / unit.
    // Every inner loop runs four independent LDS reads per step: one read per step made each
    // lane's reduction a chain of dependent LDS round trips (fc1 over Cin = 256: 16 of them; the
    // means over 16x16 planes: 16), ~5 us of the ST prologue at every batch size (r04 probe:
    // st_prologue with the SE gate skipped, profiles/r04/w)
    const int row = tid >> 4, rl = tid & 15;
    const int n4 = hw >> 2;
    if ((hw & 3) == 0 && n4 <= 16 && (n4 & (n4 - 1)) == 0) {
        // small planes (gen64's 4x4 and 8x8): one thread per channel, the plane as float4 LDS reads
        // in a per-thread rotated order (threads hw floats apart would otherwise share one bank
        // group) -- no DPP reduction chain, one round for Cin <= 512
        for (int ch = tid; ch < Cin; ch += ST_THREADS) {
            const float4* xc = reinterpret_cast<const float4*>(xs + ch * hw);
            float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            for (int i = 0; i < n4; ++i) {
                const float4 v = xc[(i + ch) & (n4 - 1)];
                acc.x += v.x;
                acc.y += v.y;
                acc.z += v.z;
                acc.w += v.w;
            }
            gate[ch] = ((acc.x + acc.y) + (acc.z + acc.w)) / (float)hw;   // channel mean (gate below)
        }
    } else {
#pragma unroll 4
        for (int ch = row; ch < Cin; ch += ST_THREADS / 16) {
            const float* xc = xs + ch * hw;
            float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f, s3 = 0.0f;
            int i = rl;
            for (; i + 48 < hw; i += 64) {
                s0 += xc[i];
                s1 += xc[i + 16];
                s2 += xc[i + 32];
                s3 += xc[i + 48];
            }
            for (; i < hw; i += 16) s0 += xc[i];
            float s = (s0 + s1) + (s2 + s3);
            s = ffc::row16_sum(s);
            if (rl == 15) gate[ch] = s / (float)hw;  // channel mean (overwritten by the gate below)
        }
    }
    __syncthreads();
    // fc1: one wave per hidden unit (64 lanes over the inputs)
    for (int j = wave; j < hid; j += ST_WAVES) {
        const float* w1 = a.w1_off >= 0 ? sm + a.w1_off + (size_t)j * Cin : a.w1 + (size_t)j * Cin;
        float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f, s3 = 0.0f;
        int k = lane;
        for (; k + 192 < Cin; k += 256) {
            s0 = fmaf(w1[k], gate[k], s0);
            s1 = fmaf(w1[k + 64], gate[k + 64], s1);
            s2 = fmaf(w1[k + 128], gate[k + 128], s2);
            s3 = fmaf(w1[k + 192], gate[k + 192], s3);
        }
        for (; k < Cin; k += 64) s0 = fmaf(w1[k], gate[k], s0);
        // the two 32-lane halves' sums (DPP + permlane16 swap), added on the scalar side
        const float hs = ffc::half_wave_sum((s0 + s1) + (s2 + s3));
        const float s = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, hs), 0)) +
                        __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, hs), 32));
        if (lane == 0) hv[j] = fmaxf(s, 0.0f);
    }
    __syncthreads();
    // fc2 + sigmoid
    const int h4 = hid >> 2;
    if (a.w2_off >= 0 && hid > 0 && (hid & 3) == 0 && h4 <= 16 && (h4 & (h4 - 1)) == 0) {
        // few hidden units (gen64: Cin / 16 = 4 .. 16): one thread per input channel k, its w2 row as
        // float4 LDS reads in a rotated order (rows hid floats apart), hv broadcast
        const float4* hv4 = reinterpret_cast<const float4*>(hv);
        for (int k = tid; k < Cin; k += ST_THREADS) {
            const float4* w2 = reinterpret_cast<const float4*>(sm + a.w2_off + k * hid);
            float s = 0.0f;
            for (int i = 0; i < h4; ++i) {
                const int q = (i + k) & (h4 - 1);
                const float4 w = w2[q], hh = hv4[q];
                s = fmaf(w.x, hh.x, s);
                s = fmaf(w.y, hh.y, s);
                s = fmaf(w.z, hh.z, s);
                s = fmaf(w.w, hh.w, s);
            }
            const float gk = 1.0f / (1.0f + expf(-s));
            gate[k] = gk;
            if (a.gate_out && sp == 0) a.gate_out[(size_t)b * Cin + k] = gk;
        }
    } else {
        // one 16-lane row per input channel k (lanes over the hidden units)
#pragma unroll 4
        for (int k = row; k < Cin; k += ST_THREADS / 16) {
            float s = 0.0f;
            if (a.w2_off >= 0) {
                const float* w2 = sm + a.w2_off + k * hid;
                for (int j = rl; j < hid; j += 16) s = fmaf(w2[j], hv[j], s);
            } else {
                for (int j = rl; j < hid; j += 16) s = fmaf(a.w2[(size_t)k * hid + j], hv[j], s);
            }
            s = ffc::row16_sum(s);
            if (rl == 15) {
                const float gk = 1.0f / (1.0f + expf(-s));   // hidden = 0: sigmoid(0) = 0.5
                gate[k] = gk;
                if (a.gate_out && sp == 0) a.gate_out[(size_t)b * Cin + k] = gk;
            }
        }
    }
    __syncthreads();
    ST_STAMP(2);

    // 3. conv1: t[o][p] = sum_k W[o][k] gate[k] x[k][p] on MFMA; lane half h carries k = 2s + h.
    //    With fewer than 4 output tiles the K range is split over the idle waves (LDS reduction).
    //    With split > 1 this workgroup takes tiles [t0, t0 + tiles) of the sample's MT x NT (the
    //    load and the SE gate are repeated per workgroup; small batches fill the CUs this way)
    const int h2 = lane >> 5, col = lane & 31;
    const int MT = Mpad / 32, NT = (hw + 31) / 32;
    const int tiles = MT * NT / a.split, t0 = sp * tiles;
    const int nsplit = tiles >= ST_WAVES ? 1 : ST_WAVES / tiles;
    const int KS = Cin / 2;
    const float* wa = a.wt_off >= 0 ? wt : a.wcT;
    auto mfma_range = [&](int mt, int nt, int s0, int s1, bool odd_tail) {
        floatx16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
        const int p = nt * 32 + col;
        const int pc = p < hw ? p : hw - 1;
        const float* ap = wa + mt * 32 + col;
        const float* xp = xs + pc;
#pragma unroll 4
        for (int s = s0; s < s1; ++s) {
            const int k = 2 * s + h2;
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ap[(size_t)k * Mpad], xp[k * hw] * gate[k], acc, 0, 0, 0);
        }
        if (odd_tail && (Cin & 1)) {  // odd Cin: last channel in slot 0, zero in slot 1
            const int k = Cin - 1;
            const float av = h2 == 0 ? ap[(size_t)k * Mpad] : 0.0f;
            const float bv = h2 == 0 ? xp[k * hw] * gate[k] : 0.0f;
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
        }
        return acc;
    };
    // split-bf16 products (ffc_internal.h split3 / mfma_split3: fp32-accurate, six bf16 MFMAs per 16 k
    // instead of eight f32 MFMAs at twice their cycles): k-block q of 16 channels, lane half h2 holds
    // channels 16q + 8 h2 + j; A from the pre-split fragments (three coalesced 16-byte loads), B = the
    // gated sample split in registers
    const int KQ = Cin >> 4;
    auto mfma_range3 = [&](int mt, int nt, int q0, int q1) {
        floatx16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
        const int p = nt * 32 + col;
        const int pc = p < hw ? p : hw - 1;
        const float* xp = xs + pc;
        const uint16_t* af = a.wc3 + (size_t)mt * KQ * 1536 + lane * 8;
#pragma unroll 2
        for (int q = q0; q < q1; ++q) {
            const uint16_t* f = af + (size_t)q * 1536;
            Split3 A;
            A.hi = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(f));
            A.mid = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(f + 512));
            A.lo = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(f + 1024));
            float xb[8];
            const int k0 = 16 * q + 8 * h2;
#pragma unroll
            for (int j = 0; j < 8; ++j) xb[j] = xp[(k0 + j) * hw] * gate[k0 + j];
            acc = mfma_split3(A, split3(xb), acc);
        }
        return acc;
    };
    const bool use3 = a.wc3 != nullptr;
    auto finish = [&](int mt, int nt, const floatx16& acc) {
        const int p = nt * 32 + col;
        const bool valid = p < hw;
        const int nv = min(32, hw - nt * 32);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int o = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h2;
            if (valid && o < c) a.t[((size_t)b * c + o) * hw + p] = acc[r];
        }
        float mean, m2;
        ffc::tile_row_stats(acc, nv, scr + wave * ffc::TILE_SCRATCH, mean, m2);
        const int o = mt * 32 + (lane >> 1);
        if ((lane & 1) == 0 && o < c) {
            float* e = st + (nt * c + o) * 3;
            e[0] = (float)nv;
            e[1] = mean;
            e[2] = m2;
        }
    };
    if (nsplit == 1) {
        for (int tl = wave; tl < tiles; tl += ST_THREADS / 64) {
            const int tile = t0 + tl, mt = tile % MT, nt = tile / MT;
            finish(mt, nt, use3 ? mfma_range3(mt, nt, 0, KQ) : mfma_range(mt, nt, 0, KS, true));
        }
    } else {
        const int tl = wave / nsplit, part = wave % nsplit, tile = t0 + tl;
        const int mt = tile % MT, nt = tile / MT;
        floatx16 acc;
        if (use3) {
            const int per = (KQ + nsplit - 1) / nsplit;
            if (tl < tiles) acc = mfma_range3(mt, nt, min(KQ, part * per), min(KQ, (part + 1) * per));
        } else {
            const int per = (KS + nsplit - 1) / nsplit;
            if (tl < tiles) acc = mfma_range(mt, nt, min(KS, part * per), min(KS, (part + 1) * per), part == 0);
        }
        if (tl < tiles && part > 0) {
#pragma unroll
            for (int r = 0; r < 16; ++r) red[(wave * 16 + r) * 64 + lane] = acc[r];
        }
        __syncthreads();
        if (tl < tiles && part == 0) {
            for (int q = 1; q < nsplit; ++q)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] += red[((wave + q) * 16 + r) * 64 + lane];
            finish(mt, nt, acc);
        }
    }
    __syncthreads();
    ST_STAMP(3);
    // one slab row per (sample, workgroup); a channel none of this workgroup's tiles covers gets
    // {0, 0, 0} (weightless in the moment sums of every consumer)
    for (int o = tid; o < c; o += ST_THREADS) {
        float nn = 0.0f, mean = 0.0f, m2 = 0.0f;
        for (int nt = 0; nt < NT; ++nt) {
            const int tile = (o >> 5) + MT * nt;
            if (tile < t0 || tile >= t0 + tiles) continue;
            const float* e = st + (nt * c + o) * 3;
            const float tot = nn + e[0];
            const float delta = e[1] - mean;
            mean += delta * (e[0] / tot);
            m2 += e[2] + delta * delta * (nn * e[0] / tot);
            nn = tot;
        }
        reinterpret_cast<float4*>(a.slab)[((size_t)b * a.split + sp) * c + o] = make_float4(nn, mean, m2, 0.0f);
    }
#ifdef FFC_TRACE
    __syncthreads();
    ST_STAMP(4);
    if (tid == 0) g_st_trace[8 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
#endif
}

// LDS plan (floats): sample, gate, hidden, tile stats, split-K partials, stats scratch, then the
// conv1 weight and the SE weights when they fit (DMA regions padded to whole 64 x 16-B groups).
struct StLayout {
    size_t bytes;
    int gate_off, hv_off, st_off, red_off, scr_off, wt_off, w1_off, w2_off;
};
size_t pad256(size_t n) { return (n + 255) / 256 * 256; }
// stage_wt = false: conv1 runs on the pre-split fragments (ffc_st_pack_a3) read from L2, so its f32
// weight is not staged (at gen64 ffc1 that copy was 64 KB of LDS-DMA per workgroup, unused)
StLayout st_layout(int Cin, int H, int W, int pool, int hid, int c, bool stage_wt = true) {
    const int h = pool ? H / 2 : H, w = pool ? W / 2 : W;
    const size_t hw = (size_t)h * w;
    const size_t nt = (hw + 31) / 32;
    const size_t Mpad = (size_t)((c + 31) & ~31);
    StLayout L{};
    size_t o = pad256((size_t)Cin * hw);
    L.gate_off = (int)o;
    o += (Cin + 3) & ~3;
    L.hv_off = (int)o;
    o += (hid + 3) & ~3;
    L.st_off = (int)o;
    o += (nt * c * 3 + 3) / 4 * 4;
    L.red_off = (int)o;
    o += ST_WAVES * 16 * 64;
    L.scr_off = (int)o;
    o += ST_WAVES * ffc::TILE_SCRATCH;
    const size_t base = o;
    const bool w12_ok = hid > 0 && ((size_t)hid * Cin) % 4 == 0;
    for (int opt = 0; opt < 3; ++opt) {   // 0: conv1 + SE weights staged, 1: conv1 only, 2: neither
        size_t q = base;
        int wt = -1, w1 = -1, w2 = -1;
        if (opt < 2 && stage_wt) {
            wt = (int)q;
            q += pad256((size_t)Cin * Mpad);
        }
        if (opt == 0) {
            if (!w12_ok) continue;
            w1 = (int)q;
            q += pad256((size_t)hid * Cin);
            w2 = (int)q;
            q += pad256((size_t)hid * Cin);
        }
        if (4 * q <= 160 * 1024) {
            L.bytes = 4 * q;
            L.wt_off = wt;
            L.w1_off = w1;
            L.w2_off = w2;
            return L;
        }
    }
    L.bytes = 0;
    return L;
}

// conv1 weight (c, Cin) row-major -> split-bf16 MFMA fragments: element
// ((mt * Cin/16 + q) * 3 + piece) * 512 + lane * 8 + j holds piece `piece` of
// W[m = 32 mt + (lane & 31)][k = 16 q + 8 (lane >> 5) + j] (zero for m >= c)
__global__ void st_pack_a3_kernel(const float* __restrict__ w, int c, int cin, uint16_t* __restrict__ out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int lane = i & 63, fr = i >> 6;
    const int KQ = cin >> 4;
    const int mt = fr / KQ, q = fr - mt * KQ;
    const int m = 32 * mt + (lane & 31), k0 = 16 * q + 8 * (lane >> 5);
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = m < c ? w[(size_t)m * cin + k0 + j] : 0.0f;
    const Split3 sp = split3(v);
    uint16_t* dst = out + (size_t)fr * 1536 + lane * 8;
    *reinterpret_cast<u32x4*>(dst) = __builtin_bit_cast(u32x4, sp.hi);
    *reinterpret_cast<u32x4*>(dst + 512) = __builtin_bit_cast(u32x4, sp.mid);
    *reinterpret_cast<u32x4*>(dst + 1024) = __builtin_bit_cast(u32x4, sp.lo);
}

}  // namespace

extern "C" size_t ffc_st_pack_a3_elems(int c, int cin) {
    if (c <= 0 || cin <= 0 || cin % 16 || c > 65536 || cin > 65536) return 0;
    return (size_t)((c + 31) / 32) * (cin / 16) * 1536;
}

extern "C" int ffc_st_pack_a3(const float* w, int c, int cin, uint16_t* out, void* stream) {
    FFC_CHECK_ARG(w && out && ffc_st_pack_a3_elems(c, cin) > 0, "ffc_st_pack_a3: bad args (Cin % 16 == 0)");
    FFC_CHECK_ARG((reinterpret_cast<uintptr_t>(out) & 15) == 0, "ffc_st_pack_a3: out must be 16-byte aligned");
    const int n = (c + 31) / 32 * (cin / 16) * 64;
    hipLaunchKernelGGL(st_pack_a3_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, w, c, cin, out, n);
    return ffc::launch_status("ffc_st_pack_a3");
}

#ifdef FFC_TRACE
extern "C" int ffc_debug_st_trace_read(void* dst, size_t bytes) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_st_trace), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

extern "C" size_t ffc_st_prologue_lds_bytes(int Cin, int H, int W, int pool, int hidden, int c) {
    if (Cin <= 0 || H <= 0 || W <= 0 || c <= 0 || hidden < 0) return 0;
    // a sample in 160 KiB of LDS has < 40960 floats: larger dims never fit (and keep the layout
    // arithmetic inside int range)
    if (Cin > 65536 || H > 65536 || W > 65536 || c > 65536 || hidden > 65536) return 0;
    if (pool && ((H | W) & 1)) return 0;
    return st_layout(Cin, H, W, pool, hidden, c).bytes;
}

extern "C" int ffc_st_prologue_split(int B, int Cin, int H, int W, int pool, int c) {
    if (B <= 0 || Cin <= 0 || H <= 0 || W <= 0 || c <= 0 || c > 65536 || H > 65536 || W > 65536) return 1;
    const long long hw = (long long)(pool ? H / 2 : H) * (pool ? W / 2 : W);
    const long long T = (long long)((c + 31) / 32) * ((hw + 31) / 32);
    // workgroups per sample: enough for one per CU (256), a divisor of the tile count
    int s = 1;
    while ((long long)B * s < 256 && T % (2 * s) == 0 && s < 8) s *= 2;
    return s;
}

extern "C" int ffc_st_prologue(const float* x, int B, int Cin, int H, int W, int pool, const float* w1,
                               const float* w2, int hidden, const float* wconv1T, int c, float* t, float* slab,
                               float* gate_out, void* stream) {
    return ffc_st_prologue_ex(x, B, Cin, H, W, pool, w1, w2, hidden, wconv1T, c, 1, t, slab, gate_out, stream);
}

extern "C" int ffc_st_prologue_ex(const float* x, int B, int Cin, int H, int W, int pool, const float* w1,
                                  const float* w2, int hidden, const float* wconv1T, int c, int split, float* t,
                                  float* slab, float* gate_out, void* stream) {
    return ffc_st_prologue_ex3(x, B, Cin, H, W, pool, w1, w2, hidden, wconv1T, nullptr, c, split, t, slab, gate_out,
                               stream);
}

extern "C" int ffc_st_prologue_ex3(const float* x, int B, int Cin, int H, int W, int pool, const float* w1,
                                   const float* w2, int hidden, const float* wconv1T, const uint16_t* wc3, int c,
                                   int split, float* t, float* slab, float* gate_out, void* stream) {
    FFC_CHECK_ARG(x && wconv1T && t && slab && B > 0, "ffc_st_prologue: bad args");
    FFC_CHECK_ARG(!wc3 || (Cin % 16 == 0 && (reinterpret_cast<uintptr_t>(wc3) & 15) == 0),
                  "ffc_st_prologue: split-bf16 conv1 fragments need Cin % 16 == 0 and 16-byte alignment");
    {
        const long long hw = (long long)(pool ? H / 2 : H) * (pool ? W / 2 : W);
        const long long T = (long long)((c + 31) / 32) * ((hw + 31) / 32);
        FFC_CHECK_ARG(split >= 1 && T % split == 0, "ffc_st_prologue: split must divide conv1's output tiles");
    }
    FFC_CHECK_ARG(hidden == 0 || (w1 && w2), "ffc_st_prologue: null SE weights");
    FFC_CHECK_ARG(ffc_st_prologue_lds_bytes(Cin, H, W, pool, hidden, c) > 0,
                  "ffc_st_prologue: sample does not fit in LDS (use se_gate + conv)");
    const StLayout L = st_layout(Cin, H, W, pool, hidden, c, wc3 == nullptr);
    const size_t lds = L.bytes;
    if (lds > 64 * 1024) {
        static std::once_flag once;
        static hipError_t err = hipSuccess;
        std::call_once(once, [] {
            err = hipFuncSetAttribute(reinterpret_cast<const void*>(st_prologue_kernel),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        });
        if (err != hipSuccess) {
            ffc::set_error(std::string("ffc_st_prologue: hipFuncSetAttribute: ") + hipGetErrorString(err));
            return FFC_E_LAUNCH;
        }
    }
    StArgs a;
    a.x = x;
    a.w1 = w1;
    a.w2 = w2;
    a.wcT = wconv1T;
    a.t = t;
    a.slab = slab;
    a.gate_out = gate_out;
    a.Cin = Cin;
    a.H = H;
    a.W = W;
    a.pool = pool;
    a.hid = hidden;
    a.c = c;
    a.gate_off = L.gate_off;
    a.hv_off = L.hv_off;
    a.st_off = L.st_off;
    a.red_off = L.red_off;
    a.scr_off = L.scr_off;
    a.wt_off = L.wt_off;
    a.w1_off = L.w1_off;
    a.w2_off = L.w2_off;
    a.split = split;
    a.wc3 = wc3;
    a.x_dma = !pool && ((size_t)Cin * H * W) % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
    if (L.w1_off >= 0 && ((reinterpret_cast<uintptr_t>(w1) | reinterpret_cast<uintptr_t>(w2)) & 15)) {
        a.w1_off = a.w2_off = -1;   // unaligned SE weights: read from global
    }
    if (L.wt_off >= 0 && (reinterpret_cast<uintptr_t>(wconv1T) & 15)) a.wt_off = -1;
    hipLaunchKernelGGL(st_prologue_kernel, dim3((unsigned)B * split), dim3(ST_THREADS), lds, (hipStream_t)stream, a);
    return ffc::launch_status("ffc_st_prologue");
}
