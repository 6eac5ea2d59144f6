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
    int wt_lds;          // conv1 weight staged in LDS
};

constexpr int ST_THREADS = 256;

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
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int Cin = a.Cin, c = a.c;
    const int h = a.pool ? a.H / 2 : a.H, w = a.pool ? a.W / 2 : a.W;
    const int hw = h * w;
    const int Mpad = (c + 31) & ~31;
    float* xs = sm;                      // [Cin][hw]
    float* gate = xs + ((Cin * hw + 3) & ~3);  // [Cin]
    float* hv = gate + ((Cin + 3) & ~3); // [hid]
    float* st = hv + ((a.hid + 3) & ~3); // [ntile][c][3]
    float* red = st + (((hw + 31) / 32) * c * 3 + 3) / 4 * 4;   // [4 waves][16][64] split-K partials
    float* scr = red + 4 * 16 * 64;      // [4 waves][32 x 33] tile-stats scratch
    float* wt = scr + 4 * ffc::TILE_SCRATCH;   // [Cin][Mpad] conv1 weight (when it fits)

#ifdef FFC_TRACE
    if (tid == 0) g_st_trace[8 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
#endif
    ST_STAMP(0);
    // 1. sample -> LDS (2x2 average pool on the way in)
    const float* xb = a.x + (size_t)b * Cin * a.H * a.W;
    if (!a.pool) {
        const int n = Cin * hw;
        if ((n & 3) == 0) {
            for (int i = tid; i < n / 4; i += ST_THREADS)
                reinterpret_cast<float4*>(xs)[i] = reinterpret_cast<const float4*>(xb)[i];
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
    if (a.wt_lds) {  // pre-transposed (Cin, Mpad) weight: plain coalesced copy
        const int n4 = Cin * Mpad / 4;
        for (int i = tid; i < n4; i += ST_THREADS)
            reinterpret_cast<float4*>(wt)[i] = reinterpret_cast<const float4*>(a.wcT)[i];
    }
    __syncthreads();
    ST_STAMP(1);

    // 2. SE gate.  Reductions run over 16-lane DPP rows (no shuffle chains): row q of the
    //    block (16 lanes, consecutive pixels / inputs: conflict-free LDS) owns one channel / unit.
    const int row = tid >> 4, rl = tid & 15;
    for (int ch = row; ch < Cin; ch += ST_THREADS / 16) {
        float s = 0.0f;
        for (int i = rl; i < hw; i += 16) s += xs[ch * hw + i];
        s = ffc::row16_sum(s);
        if (rl == 15) gate[ch] = s / (float)hw;  // channel mean (overwritten by the gate below)
    }
    __syncthreads();
    for (int j = row; j < a.hid; j += ST_THREADS / 16) {  // fc1: one 16-lane row per hidden unit
        float s = 0.0f;
        for (int k = rl; k < Cin; k += 16) s = fmaf(a.w1[(size_t)j * Cin + k], gate[k], s);
        s = ffc::row16_sum(s);
        if (rl == 15) hv[j] = fmaxf(s, 0.0f);
    }
    __syncthreads();
    float g = 0.0f;
    if (tid < Cin) {
        float s = 0.0f;
        for (int j = 0; j < a.hid; ++j) s = fmaf(a.w2[(size_t)tid * a.hid + j], hv[j], s);
        g = 1.0f / (1.0f + expf(-s));
    }
    for (int k0 = 0; k0 < Cin; k0 += ST_THREADS) {  // Cin may exceed the block
        const int k = k0 + tid;
        float gk = g;
        if (k0 > 0 && k < Cin) {
            float s = 0.0f;
            for (int j = 0; j < a.hid; ++j) s = fmaf(a.w2[(size_t)k * a.hid + j], hv[j], s);
            gk = 1.0f / (1.0f + expf(-s));
        }
        __syncthreads();
        if (k < Cin) {
            gate[k] = gk;
            if (a.gate_out) a.gate_out[(size_t)b * Cin + k] = gk;
        }
    }
    __syncthreads();
    ST_STAMP(2);

    // 3. conv1: t[o][p] = sum_k W[o][k] gate[k] x[k][p] on MFMA; lane half h carries k = 2s + h.
    //    With fewer than 4 output tiles the K range is split over the idle waves (LDS reduction).
    const int h2 = lane >> 5, col = lane & 31;
    const int MT = Mpad / 32, NT = (hw + 31) / 32;
    const int tiles = MT * NT;
    const int nsplit = tiles >= 4 ? 1 : 4 / tiles;
    const int KS = Cin / 2;
    const float* wa = a.wt_lds ? wt : a.wcT;
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
        for (int tile = wave; tile < tiles; tile += ST_THREADS / 64) {
            const int mt = tile % MT, nt = tile / MT;
            finish(mt, nt, mfma_range(mt, nt, 0, KS, true));
        }
    } else {
        const int tile = wave / nsplit, part = wave % nsplit;
        const int mt = tile % MT, nt = tile / MT;
        const int per = (KS + nsplit - 1) / nsplit;
        floatx16 acc;
        if (tile < tiles) acc = mfma_range(mt, nt, min(KS, part * per), min(KS, (part + 1) * per), part == 0);
        if (tile < tiles && part > 0) {
#pragma unroll
            for (int r = 0; r < 16; ++r) red[(wave * 16 + r) * 64 + lane] = acc[r];
        }
        __syncthreads();
        if (tile < tiles && part == 0) {
            for (int q = 1; q < nsplit; ++q)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] += red[((wave + q) * 16 + r) * 64 + lane];
            finish(mt, nt, acc);
        }
    }
    __syncthreads();
    ST_STAMP(3);
    for (int o = tid; o < c; o += ST_THREADS) {
        float nn = 0.0f, mean = 0.0f, m2 = 0.0f;
        for (int nt = 0; nt < NT; ++nt) {
            const float* e = st + (nt * c + o) * 3;
            const float tot = nn + e[0];
            const float delta = e[1] - mean;
            mean += delta * (e[0] / tot);
            m2 += e[2] + delta * delta * (nn * e[0] / tot);
            nn = tot;
        }
        reinterpret_cast<float4*>(a.slab)[(size_t)b * c + o] = make_float4(nn, mean, m2, 0.0f);
    }
#ifdef FFC_TRACE
    __syncthreads();
    ST_STAMP(4);
    if (tid == 0) g_st_trace[8 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
#endif
}

size_t st_lds(int Cin, int H, int W, int pool, int hid, int c, bool with_w) {
    const int h = pool ? H / 2 : H, w = pool ? W / 2 : W;
    const size_t hw = (size_t)h * w;
    const size_t nt = (hw + 31) / 32;
    const size_t Mpad = (size_t)((c + 31) & ~31);
    return sizeof(float) * (((Cin * hw + 3) & ~(size_t)3) + ((Cin + 3) & ~3) + ((hid + 3) & ~3) + (nt * c * 3 + 3) / 4 * 4 +
                            4 * 16 * 64 + 4 * ffc::TILE_SCRATCH + (with_w ? Cin * Mpad : 0));
}

}  // namespace

#ifdef FFC_TRACE
extern "C" int ffc_debug_st_trace_read(void* dst, size_t bytes) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_st_trace), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

extern "C" size_t ffc_st_prologue_lds_bytes(int Cin, int H, int W, int pool, int hidden, int c) {
    if (Cin <= 0 || H <= 0 || W <= 0 || c <= 0 || hidden < 0) return 0;
    if (pool && ((H | W) & 1)) return 0;
    const size_t bw = st_lds(Cin, H, W, pool, hidden, c, true);
    if (bw <= 160 * 1024) return bw;
    const size_t b = st_lds(Cin, H, W, pool, hidden, c, false);
    return b <= 160 * 1024 ? b : 0;
}

extern "C" int ffc_st_prologue(const float* x, int B, int Cin, int H, int W, int pool, const float* w1,
                               const float* w2, int hidden, const float* wconv1T, int c, float* t, float* slab,
                               float* gate_out, void* stream) {
    FFC_CHECK_ARG(x && wconv1T && t && slab && B > 0, "ffc_st_prologue: bad args");
    FFC_CHECK_ARG(hidden == 0 || (w1 && w2), "ffc_st_prologue: null SE weights");
    const size_t lds = ffc_st_prologue_lds_bytes(Cin, H, W, pool, hidden, c);
    FFC_CHECK_ARG(lds > 0, "ffc_st_prologue: sample does not fit in LDS (use se_gate + conv)");
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
    a.wt_lds = st_lds(Cin, H, W, pool, hidden, c, true) <= 160 * 1024;
    hipLaunchKernelGGL(st_prologue_kernel, dim3(B), dim3(ST_THREADS), lds, (hipStream_t)stream, a);
    return ffc::launch_status("ffc_st_prologue");
}
