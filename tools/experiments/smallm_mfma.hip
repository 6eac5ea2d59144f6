// Convolutions with very few output channels (M <= 4) on the bf16 MFMA with fp32-accurate split
// products (gfx950): the fgan128 generator's head conv7 (Conv2d k3 s1 p1, 2 x 64 -> 3 channels at
// 128x128 over conv6's deferred BN + GELU + NoiseInjection; FFC_BN_ACT(128, 3, 3, 0.5, 0, 1, 1, Tanh),
// fgan128_complete.py:484, ffc.py:89-97) and the FFC-DCGAN generator's last layer (ConvTranspose2d
// k4 s2 p1, 2 x 32 -> nc at 32x32 -> 64x64; models/ffc_generator.py:28, ffc_transpose.py:96-100).
//
// An M x N x K GEMM with M = 3 fills 3 of a 16-row MFMA tile.  The free rows carry the split
// pieces instead: with a = ah + am + al and b = bh + bm + bl (ffc_internal.h split3, exact bf16
// pieces), the six products of order <= 2 that make a*b fp32-accurate are
//     (ah + am + al) bh  +  ah (bm + bl)  +  am bm.
// v_mfma_f32_16x16x32_bf16 computes D[row][n] += sum_k A[row][k] B[k][n] over k = 8 g + j of lane
// group g = lane / 16.  Row r = 4 i + m (piece i of the weights of output channel m):
//   descriptor kind 1: B = the input's hi pieces at four taps (one per lane group, 8 channels each);
//                      row (i, m) holds W_i -> rows sum to (Wh + Wm + Wl) Xh;
//   descriptor kind 2: B = {mid, mid, lo, lo} pieces at two taps; row (0, m) holds Wh in every group
//                      (Wh (Xm + Xl)), row (1, m) Wm in the mid groups only (Wm Xm), row 2 zero.
// All descriptors accumulate into one 16x16 tile; out[m][n] = the sum of rows (0..2, m).  So a
// 16-pixel x 8-channel x 4-tap block of the conv takes 3 MFMAs (16 cycles each) where a padded
// 6-product tile takes 6 -- and the VALU of the old direct kernels (36 FMAs per input read) is gone:
// what stays on the VALU is the split (and the head's deferred transform) while the patch is staged.
//
// Per chunk of 8 input channels the patch (output tile + 1-pixel halo) is staged into an LDS image
// [piece][patch row][patch col] x 16 B (8 channels of bf16: one ds_read_b128 per B fragment, 16
// consecutive pixels = 256 contiguous bytes), double buffered; the split weights sit in LDS as
// [piece][tap][m][channel] for the whole kernel, and each compute wave keeps the chunk's A
// fragments (one per descriptor) in registers across its N-tiles (workgroup roles below).
#include "ffc_internal.h"

#include <cstdlib>
#include <mutex>
#include <set>

namespace {

constexpr int SQ_THREADS = 512;
typedef float floatx4_t __attribute__((ext_vector_type(4)));

struct SmqArgs {
    const float* x[2];
    const float* w[2];     // MODE 0: Conv2d weights (M, C_s, 3, 3)
    const float* wpack;    // MODE 1: ConvTranspose2d weights packed [C0 + C1][16 taps][4 m]
    int C[2];
    const float* bias;
    float* out;
    int B, IH, IW, M;      // input plane (MODE 0: = output plane)
    int nty, ntx;
    int act;
    float act_param;
    ffc_in_tf tf[2];
};

// Descriptor tables.  Per descriptor d and lane group g: the B piece (0 hi, 1 mid, 2 lo), the tap's
// input offset (dy, dx), the weight tap index (-1: zero A column), the accumulator (phase), the kind.
struct Desc {
    signed char piece[4], dy[4], dx[4], tap[4];
    signed char phase, kind;
};

// MODE 0, Conv2d k3 s1 p1: for each kernel row dy: kind 1 over dx = -1, 0, +1 (+ a zero group), kind 2
// over dx = -1, 0 and over dx = +1 (+ zero groups).  Weight tap = (dy + 1) * 3 + (dx + 1).
constexpr Desc kConv3[9] = {
    {{0, 0, 0, 0}, {-1, -1, -1, -1}, {-1, 0, 1, 1}, {0, 1, 2, -1}, 0, 1},
    {{1, 1, 2, 2}, {-1, -1, -1, -1}, {-1, 0, -1, 0}, {0, 1, 0, 1}, 0, 2},
    {{1, 1, 2, 2}, {-1, -1, -1, -1}, {1, 1, 1, 1}, {2, -1, 2, -1}, 0, 2},
    {{0, 0, 0, 0}, {0, 0, 0, 0}, {-1, 0, 1, 1}, {3, 4, 5, -1}, 0, 1},
    {{1, 1, 2, 2}, {0, 0, 0, 0}, {-1, 0, -1, 0}, {3, 4, 3, 4}, 0, 2},
    {{1, 1, 2, 2}, {0, 0, 0, 0}, {1, 1, 1, 1}, {5, -1, 5, -1}, 0, 2},
    {{0, 0, 0, 0}, {1, 1, 1, 1}, {-1, 0, 1, 1}, {6, 7, 8, -1}, 0, 1},
    {{1, 1, 2, 2}, {1, 1, 1, 1}, {-1, 0, -1, 0}, {6, 7, 6, 7}, 0, 2},
    {{1, 1, 2, 2}, {1, 1, 1, 1}, {1, 1, 1, 1}, {8, -1, 8, -1}, 0, 2},
};

// MODE 1, ConvTranspose2d k4 s2 p1 on the input grid: output (2 my + py, 2 mx + px) of phase (py, px) takes
// taps (ty, tx) in {0, 1}^2 with ky = py ? (ty ? 2 : 0) : (ty ? 3 : 1), input row my + dy, dy = py ? (ty ? 0 : 1)
// : (ty ? -1 : 0) (same for x).  Per phase: kind 1 over the four taps, kind 2 over ty = 0 and over ty = 1.
constexpr int ct_k(int p, int t) { return p ? (t ? 2 : 0) : (t ? 3 : 1); }
constexpr int ct_d(int p, int t) { return p ? (t ? 0 : 1) : (t ? -1 : 0); }
constexpr Desc ct_desc(int ph, int j) {
    const int py = ph >> 1, px = ph & 1;
    Desc d{};
    d.phase = (signed char)ph;
    d.kind = j == 0 ? 1 : 2;
    for (int g = 0; g < 4; ++g) {
        const int ty = j == 0 ? g >> 1 : j - 1, tx = g & 1;
        d.piece[g] = (signed char)(j == 0 ? 0 : (g < 2 ? 1 : 2));
        d.dy[g] = (signed char)ct_d(py, ty);
        d.dx[g] = (signed char)ct_d(px, tx);
        d.tap[g] = (signed char)(ct_k(py, ty) * 4 + ct_k(px, tx));
    }
    return d;
}
constexpr Desc kConvT[12] = {ct_desc(0, 0), ct_desc(0, 1), ct_desc(0, 2), ct_desc(1, 0), ct_desc(1, 1), ct_desc(1, 2),
                             ct_desc(2, 0), ct_desc(2, 1), ct_desc(2, 2), ct_desc(3, 0), ct_desc(3, 1), ct_desc(3, 2)};

#ifndef FFC_SMQ_SLOTS0
#define FFC_SMQ_SLOTS0 2
#endif
#ifndef FFC_SMQ_SLOTS1
#define FFC_SMQ_SLOTS1 4
#endif
template <int MODE>
struct SmqGeo;
template <>
struct SmqGeo<0> {
    static constexpr int T = 9, NPH = 1, ND = 9, TR = 16, TC = 64, SLOTS = FFC_SMQ_SLOTS0;
    static constexpr const Desc* desc() { return kConv3; }
};
template <>
struct SmqGeo<1> {
    static constexpr int T = 16, NPH = 4, ND = 12, TR = 8, TC = 32, SLOTS = FFC_SMQ_SLOTS1;
    static constexpr const Desc* desc() { return kConvT; }
};

template <int MODE>
struct SmqLayout {
    using G = SmqGeo<MODE>;
    static constexpr int PR = G::TR + 2, PC = G::TC + 2;        // patch rows / cols (1-pixel halo)
    static constexpr int NG = (G::TC + 4) / 2;                  // float2 column groups x0-2 .. x0+TC+1
    static constexpr int UNITS = PR * NG;                       // staging units per chunk (8 ch x 2 px)
    static constexpr int UPT = (UNITS + 255) / 256;             // per staging thread
    static constexpr int IMG = 3 * PR * PC * 16;                // bytes per image buffer
    static constexpr int CT = G::TC / 16;                       // 16-pixel column tiles per row
    static constexpr int NT = G::TR * CT;                       // N-tiles per output tile
    static constexpr int NTW = NT / 4;                          // per compute wave
    static constexpr int RSTEP = 4 / CT;                        // tile rows between a wave's N-tiles
    static_assert(NT % 4 == 0 && G::TC % 16 == 0 && 4 % CT == 0, "tile");
};

__host__ __device__ inline size_t smq_wtab_bytes(int T, int C) { return ((size_t)3 * T * 4 * C * 2 + 16 + 255) / 256 * 256; }
template <int MODE>
size_t smq_lds_bytes(int C) {
    return smq_wtab_bytes(SmqGeo<MODE>::T, C) + 2 * (size_t)SmqLayout<MODE>::IMG;
}

typedef float f2v __attribute__((ext_vector_type(2)));

// the transforms other than GELU (not on the fgan128 path; ReLU / LeakyReLU / Tanh / Sigmoid in tests)
// out of line: inlined into the unrolled staging code they would multiply its size
__device__ __attribute__((noinline)) f2v act_pair(f2v y, int act, float p) {
    return f2v{ffc::apply_act(y.x, act, p), ffc::apply_act(y.y, act, p)};
}

// sum over the four 16-lane groups of the wave, in every lane: v_permlane16_swap pairs groups (0, 1) and
// (2, 3), v_permlane32_swap the two halves (VALU lane moves; __shfl_xor is an LDS round trip each)
__device__ __forceinline__ float group_sum4(float v) {
    int iv = __builtin_bit_cast(int, v);
    const auto a = __builtin_amdgcn_permlane16_swap(iv, iv, false, false);
    v = __builtin_bit_cast(float, (int)a[0]) + __builtin_bit_cast(float, (int)a[1]);
    iv = __builtin_bit_cast(int, v);
    const auto b = __builtin_amdgcn_permlane32_swap(iv, iv, false, false);
    return __builtin_bit_cast(float, (int)b[0]) + __builtin_bit_cast(float, (int)b[1]);
}

// exact GELU on two values (as convt_smallm.hip gelu_as2: A&S 7.1.26 erf, packed VALU)
__device__ __forceinline__ f2v gelu2(f2v v) {
    const f2v z = f2v{fabsf(v.x), fabsf(v.y)} * 0.70710678118654752f;
    const f2v d = z * 0.3275911f + 1.0f;
    const f2v t = f2v{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
    f2v q = t * 1.061405429f - 1.453152027f;
    q = q * t + 1.421413741f;
    q = q * t - 0.284496736f;
    q = q * t + 0.254829592f;
    const f2v zz = -(z * z);
    const f2v e = q * t * f2v{__expf(zz.x), __expf(zz.y)};
    const f2v h = 0.5f * v * e;
    const f2v r = v - h;
    return f2v{v.x >= 0.0f ? r.x : h.x, v.y >= 0.0f ? r.y : h.y};
}

// Workgroup = 8 waves: waves 0-3 compute (one per SIMD: MFMAs fed from LDS, A fragments in registers),
// waves 4-7 stage (global loads two steps ahead, the head's deferred transform, the split, LDS stores).
// Persistent over the tiles (b, b + G, ...): the split weights are staged once per workgroup, and the
// (tile, chunk) steps form one stream -- the staging waves load the next tile's first chunk while the
// compute waves finish a tile and store its outputs.  One barrier per step.
template <int MODE, int MM, bool TF>
__global__ __launch_bounds__(SQ_THREADS) void smallm_mfma_kernel(SmqArgs a) {
    using G = SmqGeo<MODE>;
    using L = SmqLayout<MODE>;
    constexpr int T = G::T, ND = G::ND, NPH = G::NPH, TR = G::TR, TC = G::TC;
    constexpr int PR = L::PR, PC = L::PC, NG = L::NG, UPT = L::UPT, NTW = L::NTW, CT = L::CT, RSTEP = L::RSTEP;
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int C = a.C[0] + a.C[1];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool stager = wave >= 4;
    const size_t wtb = smq_wtab_bytes(T, C);
    char* wtab = lds;                                  // [piece][tap][m][c] bf16, then a 16-B zero block
    const int zero_off = 3 * T * 4 * C * 2;
    char* img = lds + wtb;
    const int ntiles = a.B * a.nty * a.ntx;
    const int nchunks = C / 8;
    const int mytiles = blockIdx.x < ntiles ? (ntiles - 1 - blockIdx.x) / gridDim.x + 1 : 0;
    const int nsteps = mytiles * nchunks;

    // ---- split weights -> LDS (units of 8 channels of one (tap, m)), by all waves
    for (int u = tid; u < T * 4 * (C / 8); u += SQ_THREADS) {
        const int c8 = u % (C / 8), tm = u / (C / 8), m = tm & 3, tap = tm >> 2;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int ci = 8 * c8 + j;
            float wv = 0.0f;
            if (m < a.M) {
                if constexpr (MODE == 0) {
                    const int s = ci < a.C[0] ? 0 : 1, c = s ? ci - a.C[0] : ci;
                    wv = a.w[s][((size_t)m * a.C[s] + c) * 9 + tap];
                } else {
                    wv = a.wpack[((size_t)ci * 16 + tap) * 4 + m];
                }
            }
            v[j] = wv;
        }
        const Split3 sp = split3(v);
        u32x4* d = reinterpret_cast<u32x4*>(wtab + ((size_t)tm * C + 8 * c8) * 2);
        const size_t pstride = (size_t)T * 4 * C * 2 / 16;   // u32x4 per piece plane
        d[0] = __builtin_bit_cast(u32x4, sp.hi);
        d[pstride] = __builtin_bit_cast(u32x4, sp.mid);
        d[2 * pstride] = __builtin_bit_cast(u32x4, sp.lo);
    }
    if (tid == 0) *reinterpret_cast<u32x4*>(wtab + zero_off) = u32x4{0u, 0u, 0u, 0u};

    auto tile_of = [&](int i, int& b, int& y0, int& x0) {   // i-th tile of this workgroup
        int t = blockIdx.x + i * gridDim.x;
        const int tx = t % a.ntx;
        t /= a.ntx;
        const int ty = t % a.nty;
        b = t / a.nty;
        y0 = ty * TR;
        x0 = tx * TC;
    };

    if (stager) {
        // ---------------- staging: unit = (patch row, float2 column group) x 8 channels
        const int sid = tid - 256;
        constexpr int NS = G::SLOTS;   // register slots: loads run NS - 1 steps ahead of the store
        f2v sv[NS][UPT][8], nz[NS][UPT];
        auto load = [&](int step, int slot) {
            int b, y0, x0;
            tile_of(step / nchunks, b, y0, x0);
            const int ci0 = 8 * (step % nchunks);
            const int s = ci0 < a.C[0] ? 0 : 1, c0 = s ? ci0 - a.C[0] : ci0;
            const float* xs = a.x[s] + ((size_t)b * a.C[s] + c0) * a.IH * a.IW;
            // without noise the noise loads read x (its weight is 0): no conditional load (a branch around
            // a load makes the compiler wait for every outstanding load there)
            const float* npl = TF && a.tf[s].noise ? a.tf[s].noise + (size_t)b * a.IH * a.IW : xs;
#pragma unroll
            for (int q = 0; q < UPT; ++q) {
                const int u = q * 256 + sid;
                const int pr = u / NG, g = u - pr * NG;
                const int iy = y0 - 1 + pr, ix = x0 - 2 + 2 * g;
                const bool ok = u < L::UNITS && (unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW;
                const size_t o = ok ? (size_t)iy * a.IW + ix : 0;
#pragma unroll
                for (int j = 0; j < 8; ++j) sv[slot][q][j] = *reinterpret_cast<const f2v*>(xs + (size_t)j * a.IH * a.IW + o);
                if constexpr (TF) nz[slot][q] = *reinterpret_cast<const f2v*>(npl + o);
            }
        };
        auto store = [&](int step, int slot, char* buf) {
            int b, y0, x0;
            tile_of(step / nchunks, b, y0, x0);
            const int ci0 = 8 * (step % nchunks);
            const int s = ci0 < a.C[0] ? 0 : 1, c0 = s ? ci0 - a.C[0] : ci0;
            // the chunk's transform parameters (uniform): scale, shift, noise weight per channel
            int mode = 0;   // 0: as stored, 1: BN + GELU (+ noise), 2: BN + other activation (+ noise)
            float sc[8], sh[8], nw[8];
            int act = 0;
            float actp = 0.0f;
            if constexpr (TF) {
                const ffc_in_tf& t = a.tf[s];
                if (t.scale) {
                    mode = t.act == FFC_ACT_GELU ? 1 : 2;
                    act = t.act;
                    actp = t.act_param;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        sc[j] = t.scale[c0 + j];
                        sh[j] = t.shift[c0 + j];
                        nw[j] = t.noise ? t.noise_w[c0 + j] : 0.0f;
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < UPT; ++q) {
                const int u = q * 256 + sid;
                const int pr = u / NG, g = u - pr * NG;
                const int iy = y0 - 1 + pr, ix = x0 - 2 + 2 * g;
                const bool inimg = u < L::UNITS && (unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW;
                f2v v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = sv[slot][q][j];
                if constexpr (TF) {
                    if (mode == 1) {
#pragma unroll
                        for (int j = 0; j < 8; ++j) v[j] = nz[slot][q] * nw[j] + gelu2(v[j] * sc[j] + sh[j]);
                    } else if (mode == 2) {
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            const f2v y = v[j] * sc[j] + sh[j];
                            v[j] = nz[slot][q] * nw[j] + act_pair(y, act, actp);
                        }
                    }
                }
                if (u < L::UNITS) {
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        const int pc = 2 * g - 1 + e;   // patch column of pixel e (patch col 0 = x0 - 1)
                        if (pc < 0 || pc >= PC) continue;
                        float v8[8];
#pragma unroll
                        for (int j = 0; j < 8; ++j) v8[j] = inimg ? v[j][e] : 0.0f;
                        const Split3 sp = split3(v8);
                        char* d = buf + (pr * PC + pc) * 16;
                        *reinterpret_cast<u32x4*>(d) = __builtin_bit_cast(u32x4, sp.hi);
                        *reinterpret_cast<u32x4*>(d + PR * PC * 16) = __builtin_bit_cast(u32x4, sp.mid);
                        *reinterpret_cast<u32x4*>(d + 2 * PR * PC * 16) = __builtin_bit_cast(u32x4, sp.lo);
                    }
                }
            }
        };
        if (nsteps == 0) return;
        const int last = nsteps - 1;
#pragma unroll
        for (int u = 0; u < NS; ++u) load(min(u, last), u);
#ifndef FFC_SMQ_NOSTAGE
        store(0, 0, img);
#endif
        __syncthreads();
        // period s: step s + NS's loads go out into slot s % NS (its step s was stored one period ago),
        // step s + 1 is transformed, split and stored into buffer (s + 1) & 1 while the compute waves read
        // buffer s & 1.  Slot indices are compile-time (the loop runs NS periods per iteration), and the
        // loads are issued in every period, clamped to the last step: a conditional issue makes the
        // compiler wait for all outstanding loads (vmcnt(0)) at the store, exposing a load latency per step.
        for (int s0 = 0; s0 < nsteps; s0 += NS) {
#pragma unroll
            for (int h = 0; h < NS; ++h) {
                const int s = s0 + h;
                if (h > 0 && s >= nsteps) break;
                load(min(s + NS, last), h);
#ifndef FFC_SMQ_NOSTAGE
                if (s + 1 < nsteps) store(s + 1, (h + 1) % NS, img + ((s + 1) & 1) * L::IMG);
#endif
                __syncthreads();
            }
        }
        return;
    }

    // ---------------- compute waves
    const int arow = lane & 15, ag = lane >> 4, ai = arow >> 2, am = arow & 3;
    int aoff[ND];
#pragma unroll
    for (int d = 0; d < ND; ++d) {
        const Desc& D = G::desc()[d];
        const int tap = D.tap[ag];
        const bool zero = tap < 0 || am >= MM || ai == 3 || (D.kind == 2 && (ai == 2 || (ai == 1 && D.piece[ag] != 1)));
        aoff[d] = zero ? -1 : ((ai * T + tap) * 4 + am) * C * 2;
    }
    // B-fragment byte offsets: N-tile t of wave w is tile row w / CT + t * RSTEP, column tile w % CT
    const int bn = lane & 15, bg = lane >> 4;
    const int bbase = ((wave / CT + 1) * PC + (wave % CT) * 16 + bn + 1) * 16;
    int doff[ND];
#pragma unroll
    for (int d = 0; d < ND; ++d) {
        const Desc& D = G::desc()[d];
        doff[d] = bbase + ((D.piece[bg] * PR + D.dy[bg]) * PC + D.dx[bg]) * 16;
    }
    floatx4_t acc[NTW][NPH];
#pragma unroll
    for (int t = 0; t < NTW; ++t)
#pragma unroll
        for (int p = 0; p < NPH; ++p) acc[t][p] = floatx4_t{0.f, 0.f, 0.f, 0.f};
    const float ap = a.act_param;
    const int sm = lane >> 4;
    const float bv = a.bias && sm < a.M ? a.bias[sm] : 0.0f;

    __syncthreads();
    for (int s = 0; s < nsteps; ++s) {
        const int k = s % nchunks;
        const char* cur = img + (s & 1) * L::IMG;
        bf16x8 af[ND];
#pragma unroll
        for (int d = 0; d < ND; ++d)
            af[d] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(wtab + (aoff[d] < 0 ? zero_off : aoff[d] + 16 * k)));
        // B fragments of N-tile t + 1 are read while N-tile t's MFMAs run
        bf16x8 bq[2][ND];
#pragma unroll
        for (int d = 0; d < ND; ++d) bq[0][d] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(cur + doff[d]));
#pragma unroll
        for (int t = 0; t < NTW; ++t) {
            if (t + 1 < NTW) {
#pragma unroll
                for (int d = 0; d < ND; ++d)
                    bq[(t + 1) & 1][d] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(cur + doff[d] + (t + 1) * RSTEP * PC * 16));
            }
#pragma unroll
            for (int d = 0; d < ND; ++d) {
                const Desc& D = G::desc()[d];
#ifndef FFC_SMQ_NOMFMA
                acc[t][D.phase] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[d], bq[t & 1][d], acc[t][D.phase], 0, 0, 0);
#else
                acc[t][D.phase][0] += __builtin_bit_cast(float, __builtin_bit_cast(u32x4, bq[t & 1][d])[0] & 1u);
#endif
            }
            if (t + 1 < NTW) __builtin_amdgcn_sched_group_barrier(0x100, ND, 0);   // next tile's DS reads first
            __builtin_amdgcn_sched_group_barrier(0x8, ND, 0);                      // then this tile's MFMAs
            __builtin_amdgcn_sched_barrier(0);
        }
        if (k == nchunks - 1) {
            // epilogue of the finished tile: out[m][n] = sum of rows (i, m), i = 0..2 (lane groups 0..2,
            // register m); lane group g stores output channel m = g
            int b, y0, x0;
            tile_of(s / nchunks, b, y0, x0);
#pragma unroll
            for (int t = 0; t < NTW; ++t) {
                const int r = wave / CT + t * RSTEP, c = (wave % CT) * 16 + bn;
#pragma unroll
                for (int p = 0; p < NPH; ++p) {
                    float o[4];
#pragma unroll
                    for (int m = 0; m < 4; ++m) o[m] = group_sum4(acc[t][p][m]);
                    acc[t][p] = floatx4_t{0.f, 0.f, 0.f, 0.f};
                    float v = sm == 0 ? o[0] : sm == 1 ? o[1] : sm == 2 ? o[2] : o[3];
                    v = ffc::apply_act(v + bv, a.act, ap);
                    if (sm < a.M) {
                        if constexpr (MODE == 0) {
                            const int oy = y0 + r, ox = x0 + c;
                            if (oy < a.IH && ox < a.IW) a.out[(((size_t)b * a.M + sm) * a.IH + oy) * a.IW + ox] = v;
                        } else {
                            const int my = y0 + r, mx = x0 + c;
                            const int OH = 2 * a.IH, OW = 2 * a.IW;
                            if (my < a.IH && mx < a.IW)
                                a.out[(((size_t)b * a.M + sm) * OH + 2 * my + (p >> 1)) * OW + 2 * mx + (p & 1)] = v;
                        }
                    }
                }
            }
        }
        __syncthreads();
    }
}

template <int MODE>
using SmqKernel = void (*)(SmqArgs);

template <int MODE, bool TF>
SmqKernel<MODE> pick(int M) {
    switch (M) {
        case 1: return smallm_mfma_kernel<MODE, 1, TF>;
        case 2: return smallm_mfma_kernel<MODE, 2, TF>;
        case 3: return smallm_mfma_kernel<MODE, 3, TF>;
        case 4: return smallm_mfma_kernel<MODE, 4, TF>;
    }
    return nullptr;
}

// one workgroup per CU (LDS and registers allow no second one), never more than the tiles
int persistent_grid(int ntiles) {
    static int cus = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return 256;
        return n > 0 ? n : 256;
    }();
    return ntiles < cus ? ntiles : cus;
}

int raise(const void* k, const char* what) {
    static std::mutex mu;
    static std::set<const void*> done;
    std::lock_guard<std::mutex> g(mu);
    if (done.count(k)) return FFC_OK;
    if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess) {
        ffc::set_error(std::string(what) + ": hipFuncSetAttribute failed");
        return FFC_E_LAUNCH;
    }
    done.insert(k);
    return FFC_OK;
}

// Off by default (FFC_SMALLM_MFMA=1 turns it on): measured slower than the VALU kernels on MI355X
// (profiles/r03/s2c): fgan128 B = 512 head 1.82 -> 2.42 ms, gen64 last ConvT 43 -> 60 us.  The head's
// deferred BN + GELU + noise transform and the split stay on the VALU (~23 instructions per staged
// element, two of them 8-cycle transcendentals), and every v_mfma_f32_16x16x32_bf16 holds its SIMD's
// vector issue for 8 of its 16 cycles (MI355X_MICROARCH.md, issue-cost row): the staging waves run at
// about half rate beside the compute waves (compute alone, staging skipped: 1.07 ms).  The ConvT
// (no transform) is bound by its per-step overheads (A-fragment reads, one barrier per 8 channels).
bool enabled() {
    static const bool on = [] {
        const char* e = std::getenv("FFC_SMALLM_MFMA");
        return e && e[0] == '1';
    }();
    return on;
}

}  // namespace

namespace ffc {

// Head conv (Conv2d k3 s1 p1) on the MFMA; returns 1 when the shape is not handled here (the VALU
// kernel runs instead), else FFC_OK / an error code
int smallm_mfma_conv3(const float* x0, int C0, const float* w0, const float* x1, int C1, const float* w1,
                      const float* bias, int B, int H, int W, int M, float* out, int act, float act_param,
                      const ffc_in_tf* tf0, const ffc_in_tf* tf1, void* stream) {
    const int c1 = x1 ? C1 : 0;
    if (!enabled() || M < 1 || M > 4 || C0 % 8 || c1 % 8 || W % 2 ||
        (reinterpret_cast<uintptr_t>(x0) & 7) || (x1 && (reinterpret_cast<uintptr_t>(x1) & 7)))
        return 1;
    const size_t lds = smq_lds_bytes<0>(C0 + c1);
    if (lds > 160 * 1024) return 1;
    SmqArgs a{};
    a.x[0] = x0;
    a.x[1] = x1 ? x1 : x0;
    a.w[0] = w0;
    a.w[1] = x1 ? w1 : w0;
    a.C[0] = C0;
    a.C[1] = c1;
    a.bias = bias;
    a.out = out;
    a.B = B;
    a.IH = H;
    a.IW = W;
    a.M = M;
    a.nty = (H + SmqGeo<0>::TR - 1) / SmqGeo<0>::TR;
    a.ntx = (W + SmqGeo<0>::TC - 1) / SmqGeo<0>::TC;
    a.act = act;
    a.act_param = act_param;
    const ffc_in_tf none = {nullptr, nullptr, 0, 0.0f, nullptr, nullptr};
    a.tf[0] = tf0 ? *tf0 : none;
    a.tf[1] = (x1 && tf1) ? *tf1 : none;
    for (int s = 0; s < 2; ++s)
        if (a.tf[s].noise && (reinterpret_cast<uintptr_t>(a.tf[s].noise) & 7)) return 1;
    const bool tf = a.tf[0].scale || a.tf[1].scale;
    SmqKernel<0> k = tf ? pick<0, true>(M) : pick<0, false>(M);
    const int rc = raise(reinterpret_cast<const void*>(k), "ffc_conv3x3_smallm (mfma)");
    if (rc) return rc;
    hipLaunchKernelGGL(k, dim3(persistent_grid(B * a.nty * a.ntx)), dim3(SQ_THREADS), lds, (hipStream_t)stream, a);
    return launch_status("ffc_conv3x3_smallm (mfma)");
}

// Last ConvT (k4 s2 p1) on the MFMA from the packed weights of ffc_convt_smallm_pack; 1 = not handled
int smallm_mfma_convt(const float* x0, int C0, const float* x1, int C1, const float* wpack, const float* bias,
                      int B, int IH, int IW, int M, float* out, int act, float act_param, void* stream) {
    const int c1 = x1 ? C1 : 0;
    if (!enabled() || M < 1 || M > 4 || C0 % 8 || c1 % 8 || IW % 2 ||
        (reinterpret_cast<uintptr_t>(x0) & 7) || (x1 && (reinterpret_cast<uintptr_t>(x1) & 7)))
        return 1;
    const size_t lds = smq_lds_bytes<1>(C0 + c1);
    if (lds > 160 * 1024) return 1;
    SmqArgs a{};
    a.x[0] = x0;
    a.x[1] = x1 ? x1 : x0;
    a.wpack = wpack;
    a.C[0] = C0;
    a.C[1] = c1;
    a.bias = bias;
    a.out = out;
    a.B = B;
    a.IH = IH;
    a.IW = IW;
    a.M = M;
    a.nty = (IH + SmqGeo<1>::TR - 1) / SmqGeo<1>::TR;
    a.ntx = (IW + SmqGeo<1>::TC - 1) / SmqGeo<1>::TC;
    a.act = act;
    a.act_param = act_param;
    SmqKernel<1> k = pick<1, false>(M);
    const int rc = raise(reinterpret_cast<const void*>(k), "ffc_convt_k4s2_smallm (mfma)");
    if (rc) return rc;
    hipLaunchKernelGGL(k, dim3(persistent_grid(B * a.nty * a.ntx)), dim3(SQ_THREADS), lds, (hipStream_t)stream, a);
    return launch_status("ffc_convt_k4s2_smallm (mfma)");
}

}  // namespace ffc
