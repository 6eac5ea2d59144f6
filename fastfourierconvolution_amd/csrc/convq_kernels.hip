// Stride-2 transposed convolution as an implicit GEMM with the operands pre-split for the
// fp32-accurate bf16 MFMA products (gfx950) — the local-branch hot path of FFCTranspose
// (layers/ffc/ffc_transpose.py:79-86, ConvTranspose2d k4 s2 p1) with SpectralTransform.conv2
// (spectral_transform.py:70-71,108) folded in as a 1x1 segment at the output resolution.
//
// Why a second patch kernel (convp_kernels.hip keeps the f32-MFMA and pooled/strided paths):
// the split-bf16 products need every fp32 operand split into three exact bf16 pieces (hi, mid,
// lo: ffc_internal.h split3).  convp splits each B fragment in registers at every use, and every
// input element is used by 16 (phase, tap) fragments of a ConvT k4 s2 — ~11 VALU instructions
// per MFMA (profiles/r01j/pmc_sq_convp.txt).  Here each input element is split ONCE per
// workgroup, while it is staged:
//   * staging (global -> registers -> split -> LDS): a unit = 8 consecutive channels of one patch
//     pixel, loaded as 8 fp32 values one chunk ahead (in flight under the current chunk's MFMAs),
//     split, stored as three bf16x8 pieces with ds_write_b128 into the LDS image
//     [half h][patch pixel][piece] (48 bytes per pixel-half: the three reads of a fragment are one
//     address + immediate offsets 0/16/32, and 16 consecutive pixels hit 16 distinct bank slots);
//   * K order inside a segment is (16-channel chunk, tap, channel): a B fragment (lane = pixel n,
//     half h = 8 channels) is three ds_read_b128, no VALU;
//   * A (packed weights, same K order) is pre-split into three bf16 planes (ffc_split_bf16) and
//     loaded as three 16-byte loads per (k16 step, M-tile).
// The 1x1 segment at the output resolution (conv2) has no reuse across phases or taps, so its B
// fragments are read straight from global memory and split in registers ("direct" segment).
//
// Workgroup = 8 waves, warp-specialised: waves 0-3 compute the 4 phases (py, px) of a pixel block
// of NS samples x TR x TC phase-grid pixels (32*NTW pixels) -- wave w: MT M-tiles of 32 output
// channels x NTW N-tiles of 32 pixels of phase w, MFMAs fed from LDS and registers only -- while
// waves 4-7 stage the next chunk (global loads, split, LDS stores) into the other buffer; one
// barrier per chunk.  Each SIMD holds one computing and one staging wave, so the matrix pipe
// is never shared and the staging latency is off the MFMA path.  The compute waves also load
// A for the chunk at its start (tap 0's A one chunk ahead).  Epilogue (bias, addend, BN partial
// slab rows [block*4 + wave], activation) as in convp.
#include "ffc_internal.h"

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <tuple>

namespace {

constexpr int QTHREADS = 512;   // 4 compute waves + 4 staging waves
#ifndef FFC_CONVQ_WPE
#define FFC_CONVQ_WPE
#endif
#ifndef FFC_CONVQ_SLOTS
#define FFC_CONVQ_SLOTS 2
#endif
constexpr int QSLOTS = FFC_CONVQ_SLOTS;   // staging register slots (chunks in flight + the one being stored)
static_assert(QSLOTS >= 2 && QSLOTS <= 6, "convq staging slots");

struct ConvQArgs {
    ffc_convp_job jobs[2];
    const int4* tiles;
    int ebuf;                  // bytes per LDS buffer (multiple of 256)
    int ksplit;                // K splits per output tile (1: no split)
    float* part;               // ksplit > 1: per (slot, split, wave) fragment partial sums
    int ntiles;                // rows of the tile table (the grid may be smaller: persistent workgroups)
};

typedef __attribute__((address_space(3))) void* lptr_t;


#ifdef FFC_TRACE_Q
// Diagnostic build only (tools/trace_convq.py): per workgroup 16 u64:
// [0] realtime start [1] realtime end (compute wave 0) [2] HW_ID | XCC_ID << 32
// compute wave 0 cycles: [3] barrier waits [4] A issue + B tap-0 read [5] MFMA taps [6] direct segs
// [7] epilogue [8] total; staging wave 4 cycles: [9] loads (issue -> data) [10] split + LDS store
// [11] barrier waits [12] total; [13] chunks
__device__ unsigned long long g_ffc_trace_q[16 * 16384];
#define QSTAMP(t)                                                                           \
    do {                                                                                    \
        __builtin_amdgcn_sched_barrier(0);                                                  \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");          \
        __builtin_amdgcn_sched_barrier(0);                                                  \
    } while (0)
#endif

__device__ __forceinline__ u32x4 lds_read16(const char* base, int off) {
    return *reinterpret_cast<const u32x4*>(base + off);
}

// Pixel geometry of lane `lane` of compute wave `wave` (= phase) in pixel block pb: per N-tile the
// sample / phase-grid row / column inside the block and whether the pixel exists.
template <int NTW>
struct QGeom {
    int b0, r0, c0;
    int pns[NTW], pr_[NTW], pc_[NTW];
    bool pv[NTW];
};

template <int NTW>
__device__ __forceinline__ QGeom<NTW> q_geometry(const ffc_convp_job& J, int wave, int lane, int pb) {
    QGeom<NTW> g;
    const ffc_convp_phase& P = J.ph[wave];
    const int NS = J.NS, TR = J.TR, TC = J.TC, TRC = TR * TC;
    const int bs = pb / (J.nrb * J.ncb);
    const int prem = pb - bs * J.nrb * J.ncb;
    const int rb = prem / J.ncb, cb = prem - rb * J.ncb;
    g.b0 = bs * NS;
    g.r0 = rb * TR;
    g.c0 = cb * TC;
    const int cl = lane & 31;
    // q / TRC and rem / TC for q < 32 * NTW <= 128 through a reciprocal: (q + 0.5) / d stays >= 0.5 / d
    // >= 1/256 away from every integer and the approximate reciprocal is off by < 2^-16 there, so the
    // truncation is exact (the generic i32 division is ~30 instructions per quotient)
    const float rTRC = __builtin_amdgcn_rcpf((float)TRC), rTC = __builtin_amdgcn_rcpf((float)TC);
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) {
        const int q = nt * 32 + cl;
        const int ns = (int)(((float)q + 0.5f) * rTRC);
        const int rem = q - ns * TRC;
        const int r = (int)(((float)rem + 0.5f) * rTC), c = rem - r * TC;
        g.pns[nt] = ns;
        g.pr_[nt] = r;
        g.pc_[nt] = c;
        g.pv[nt] = ns < NS && g.b0 + ns < J.B && g.r0 + r < P.PH && g.c0 + c < P.PW;
    }
    return g;
}

// The epilogues apply only the piecewise-linear activations (identity, ReLU, LeakyReLU) as
// v > 0 ? v : v * slope: one code path instead of an unrolled store loop per activation (the kernel
// was ~200 KB of code, most of it epilogue variants run once per tile).  Tanh / Sigmoid / GELU run
// as a separate in-place pass after the launch (ffc_convq_forward_split; no model layer on this
// kernel uses them: BN follows the convolution, or the layer runs on convt_smallm).
__device__ __forceinline__ float q_slope(const ffc_convp_job& J) {
    return J.act == FFC_ACT_RELU ? 0.0f : J.act == FFC_ACT_LEAKY_RELU ? J.act_param : 1.0f;
}
__device__ __forceinline__ float q_act(float v, float slope) { return v > 0.0f ? v : v * slope; }

// one wave's fragments as MT x NTW x 4 coalesced floatx4 rows of 64 lanes
template <int MT, int NTW>
__device__ __forceinline__ void store_partial(float* dst, int lane, const floatx16 (&acc)[MT][NTW]) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt)
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4) {
                const floatx4 v = {acc[mt][nt][4 * r4], acc[mt][nt][4 * r4 + 1], acc[mt][nt][4 * r4 + 2],
                                   acc[mt][nt][4 * r4 + 3]};
                *reinterpret_cast<floatx4*>(dst + ((mt * NTW + nt) * 4 + r4) * 256 + lane * 4) = v;
            }
}

// The job fields an epilogue uses, copied out of the kernel-argument struct: the compiler cannot
// tell that the output / slab stores leave the argument memory alone, so every field read through J
// after a store was a fresh s_load + s_waitcnt lgkmcnt(0) -- per stored element (r04 ISA; ~6K
// cycles of a tile's epilogue).
struct QEpi {
    float* out;
    const float* bias;
    const float* addend;
    float* stats;
    int M, B, OH, OW;
    float slope;
};
__device__ __forceinline__ QEpi q_epi(const ffc_convp_job& J) {
    QEpi e;
    e.out = J.out;
    e.bias = J.bias;
    e.addend = J.addend;
    e.stats = J.stats;
    e.M = J.M;
    e.B = J.B;
    e.OH = J.OH;
    e.OW = J.OW;
    e.slope = q_slope(J);
    return e;
}

// BN partial slab rows [pb * 4 + wave] of one compute wave's fragments (channels mbase + (r & 3) +
// 8 (r >> 2)): {count, mean, M2} over the wave's valid pixels
template <int NTW>
__device__ __forceinline__ void q_stats(const QEpi& E, int wave, int cl, int pb, int mbase, const bool (&pv)[NTW],
                                        const floatx16 (&tacc)[NTW]) {
    float cntl = 0.0f;
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) cntl += pv[nt] ? 1.0f : 0.0f;
    const float cnt = ffc::half_wave_sum(cntl);
    float4* stp = reinterpret_cast<float4*>(E.stats) + ((size_t)pb * 4 + wave) * E.M;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int m = mbase + (r & 3) + 8 * (r >> 2);
        float sm = 0.0f;
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) sm += pv[nt] ? tacc[nt][r] : 0.0f;
        const float mean = cnt > 0.0f ? ffc::half_wave_sum(sm) / cnt : 0.0f;
        float q = 0.0f;
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) {
            const float d = pv[nt] ? tacc[nt][r] - mean : 0.0f;
            q += d * d;
        }
        const float m2 = ffc::half_wave_sum(q);
        if (cl == 0 && m < E.M) stp[m] = make_float4(cnt, mean, m2, 0.0f);
    }
}

// Epilogue of one compute wave (phase `wave`) of output tile (pb, m0): bias / addend, the BN partial
// slab rows [pb * 4 + wave], activation, scattered stores
template <int MT, int NTW>
__device__ __forceinline__ void convq_epilogue(const ffc_convp_job& J, int wave, int lane, int pb, int m0,
                                               floatx16 (&acc)[MT][NTW]) {
    const QGeom<NTW> g = q_geometry<NTW>(J, wave, lane, pb);
    const ffc_convp_phase& P = J.ph[wave];
    const QEpi E = q_epi(J);
    const int py = P.py, px = P.px;
    const int h = lane >> 5, cl = lane & 31;
    const size_t plane = (size_t)E.OH * E.OW;
    long long obase[NTW];   // per N-tile: element offset of (sample, channel 0, pixel)
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt)
        obase[nt] = (long long)(g.b0 + g.pns[nt]) * E.M * (long long)plane +
                    ((g.r0 + g.pr_[nt]) * 2 + py) * E.OW + ((g.c0 + g.pc_[nt]) * 2 + px);
    // full tile: all channels below M and every lane's pixels valid (wave-uniform); then the byte
    // offset of each lane's element from the tile's (first sample, channel m) row fits 32 bits
    // (checked on the host: NS * M * OH * OW * 4 < 2^32)
    bool allv = m0 + 32 * MT <= E.M;
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) allv = allv && g.pv[nt];
    const bool full = __builtin_amdgcn_ballot_w64(allv) == ~0ull;
    unsigned voff[NTW];
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) {
        voff[nt] = ((unsigned)g.pns[nt] * (unsigned)E.M * (unsigned)plane + (unsigned)(4 * h) * (unsigned)plane +
                    (unsigned)(((g.r0 + g.pr_[nt]) * 2 + py) * E.OW + ((g.c0 + g.pc_[nt]) * 2 + px))) * 4u;
        asm volatile("" : "+v"(voff[nt]));   // computed once, kept (not re-derived at every store)
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        floatx16 (&tacc)[NTW] = acc[mt];
        const int mbase = m0 + 32 * mt + 4 * h;
        if (E.bias || E.addend) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = mbase + (r & 3) + 8 * (r >> 2);
                if (m >= E.M) continue;
                const float bv = E.bias ? E.bias[m] : 0.0f;
#pragma unroll
                for (int nt = 0; nt < NTW; ++nt) {
                    float v = tacc[nt][r] + bv;
                    if (E.addend && g.pv[nt]) v += E.addend[obase[nt] + (long long)m * plane];
                    tacc[nt][r] = v;
                }
            }
        }
        if (E.stats) q_stats<NTW>(E, wave, cl, pb, mbase, g.pv, tacc);
        if (full) {
            // every pixel and channel of the fragments exists: no per-element masks, the channel's
            // row offset on the scalar side (saddr form: uniform base + the lane's 32-bit offset)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                float* sb = E.out + ((size_t)g.b0 * E.M + m0 + 32 * mt + (r & 3) + 8 * (r >> 2)) * plane;
#pragma unroll
                for (int nt = 0; nt < NTW; ++nt) {
                    *reinterpret_cast<float*>(reinterpret_cast<char*>(sb) + voff[nt]) = q_act(tacc[nt][r], E.slope);
                }
            }
            continue;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = mbase + (r & 3) + 8 * (r >> 2);
            if (m < E.M) {
#pragma unroll
                for (int nt = 0; nt < NTW; ++nt)
                    if (g.pv[nt]) E.out[obase[nt] + (long long)m * plane] = q_act(tacc[nt][r], E.slope);
            }
        }
    }
}

// One output tile (one row of the tile table) of one workgroup; returns when the tile is done (the
// staging waves after their last barrier of the tile, the compute waves after the epilogue).  Every
// wave of the workgroup runs the same tiles, so the barrier counts match tile by tile.
// PX pixels per staging unit (4, 2 or 1): a unit = PX consecutive pixels x 8 channels, loaded as 8
// PX-float buffer loads (one per channel), split and stored pixel by pixel.  Small tiles (a few
// patch rows per chunk: the per-rank batches of strong scaling) have far fewer 4-pixel units than
// staging threads, and one unit's loads + split + stores are the chunk's staging chain; PX = 1 runs
// the same work on 4x the threads (host: the smallest PX whose units fit the 256 staging threads).
typedef float floatx2 __attribute__((ext_vector_type(2)));
template <int PX>
struct StageVec {
    float v[PX];
};
template <int PX>
__device__ __forceinline__ StageVec<PX> stage_ld(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    StageVec<PX> r;
    if constexpr (PX == 4) {
        const floatx4 q = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
        r.v[0] = q[0]; r.v[1] = q[1]; r.v[2] = q[2]; r.v[3] = q[3];
    } else if constexpr (PX == 2) {
        const floatx2 q = __builtin_bit_cast(floatx2, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0));
        r.v[0] = q[0]; r.v[1] = q[1];
    } else {
        r.v[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, 0));
    }
    return r;
}

template <int MT, int NTW, int SL = QSLOTS, int PX = 4>
__device__ __forceinline__ void convq_tile(const ConvQArgs& args, const int tix, char* lds) {
    static_assert(SL >= 2 && SL <= 6, "convq staging slots");
    static_assert(PX == 1 || PX == 2 || PX == 4, "pixels per staging unit");
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave_id = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool stager = wave_id >= 4;
    const int wave = wave_id & 3;            // compute waves: the phase
    const int stid = tid - 256;              // staging waves: unit slot 0..255
    const int h = lane >> 5, cl = lane & 31;
    const int4 tile = args.tiles[tix];
    const int ji = __builtin_amdgcn_readfirstlane(tile.x);
    const int m0 = __builtin_amdgcn_readfirstlane(tile.y);
    const int pb = __builtin_amdgcn_readfirstlane(tile.z);
    const int tw = __builtin_amdgcn_readfirstlane(tile.w);
    const int ks = tw & 7, slot = tw >> 3;   // K split of this workgroup, output tile slot
    const int nsplit = args.ksplit;
    const ffc_convp_job& J = args.jobs[ji];
    const ffc_convp_phase& P = J.ph[wave];
    const int ebuf = args.ebuf;

    const int NS = J.NS, TR = J.TR, TC = J.TC;
    const int bs = pb / (J.nrb * J.ncb);
    const int prem = pb - bs * J.nrb * J.ncb;
    const int rb = prem / J.ncb, cb = prem - rb * J.ncb;
    const int b0 = bs * NS, r0 = rb * TR, c0 = cb * TC;
    const int TRC = TR * TC;
    const int nseg = J.nseg;

    // this lane's pixel of each N-tile (q_geometry) is recomputed where it is needed (a segment
    // change, the direct segments, the epilogue) rather than held in registers through the K loop

    floatx16 acc[MT][NTW];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.0f;

#ifdef FFC_TRACE_Q
    const unsigned long long tq_rt0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long tq_0, tq_a, tq_b, tq_c, tq_d, tq_bar = 0, tq_A = 0, tq_mf = 0;
    QSTAMP(tq_0);
#endif
    // A in fragment order (ffc_convq_pack_a3): fragment (M-tile, 16-k step) = three 1 KiB planes, lane l's
    // 16 bytes at l * 16: one fully coalesced dwordx4 per (fragment, piece)
    const int ksteps = P.Kpad >> 4;
    const uint16_t* __restrict__ Afrag = J.A3 + 3 * P.a_off + (size_t)(m0 >> 5) * ksteps * 1536 + lane * 8;
    auto load_A = [&](int k, Split3 (&a)[MT]) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const uint16_t* f = Afrag + ((size_t)mt * ksteps + (k >> 4)) * 1536;
            a[mt].hi = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(f));
            a[mt].mid = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(f + 512));
            a[mt].lo = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(f + 1024));
        }
    };

    // ---------------- staged segments: chunks of 16 channels, patch image in LDS
    // The patch rows are staged in aligned 4-pixel groups from xa = ix0 & ~3 (IW % 4 == 0: a group is
    // wholly inside or outside the row): one staging unit = (sample, patch row, group, channel
    // half) = 8 channels x 4 pixels = 8 coalesced 16-byte loads; pixel e of the group is split and
    // stored at image column 4 g + e.  Image pixel (ns, row, col) of channel half h sits at
    // 48 * ((h * NS + ns) * qsample + row * qrow + col) bytes; the lane pixel (pc) of the compute
    // side is image column pc * mult_x + xoff, xoff = ix0 - xa.
    // The loads go through a buffer descriptor of the segment (ffc::buf_rsrc): a lane's byte offset of
    // its unit (sample, pixel group, channel half) is fixed for the whole segment and the chunk's
    // channel offsets are wave-uniform (SGPR soffset), so a chunk's 8 loads need no per-lane address
    // arithmetic; units outside the batch / input / unit range load at offset OOB and read zeros
    // (no select at store time), and the per-chunk state lives in registers (a kernel-argument load
    // per chunk made the wave wait for its own LDS stores: s_waitcnt lgkmcnt(0) covers both).
    struct {
        __amdgpu_buffer_rsrc_t rs;
        unsigned voff;             // byte offset of the unit's first channel at its group's first pixel (OOB: none)
        unsigned cstride;          // bytes per channel plane
        int C, Cpad, cfull;        // cfull: C % 16 == 0 (every channel of every chunk exists)
        int hu8;                   // 8 * the unit's channel half
        int wb;                    // LDS byte offset of the group's first pixel inside a buffer (-1: none)
    } st;
    auto stage_setup = [&](int s) {
        const ffc_convp_seg& S = J.seg[s];
        const int IHW = S.IH * S.IW;
        st.rs = ffc::buf_rsrc(S.x, (unsigned long long)J.B * S.C * IHW * 4);
        st.C = S.C;
        st.Cpad = S.Cpad;
        st.cfull = (S.C & 15) == 0;
        st.cstride = (unsigned)IHW * 4u;
        const int PR = S.PR, G = S.PC / PX, QR = S.qrow, QS = S.qsample;
        const int ngrp = NS * PR * G;
        const int nunits = 2 * ngrp;
        const int iy0 = r0 * S.mult_y + S.org_y;
        const int xa = (c0 * S.mult_x + S.org_x) & ~3;
        const int n = stid;
        const int hu = n >= ngrp ? 1 : 0;
        const int q = n - hu * ngrp;
        const int g = q % G, q1 = q / G;
        const int pr = q1 % PR, ns = q1 / PR;
        const int b = b0 + ns, iy = iy0 + pr, ix = xa + PX * g;
        const bool ok = n < nunits && b < J.B && (unsigned)iy < (unsigned)S.IH && (unsigned)ix < (unsigned)S.IW;
        st.voff = ok ? (unsigned)(((b * S.C + 8 * hu) * IHW + iy * S.IW + ix) * 4) : ffc::OOB;
        st.hu8 = 8 * hu;
        st.wb = n < nunits ? ((hu * NS + ns) * QS + pr * QR + PX * g) * 48 : -1;
    };
    auto stage_load = [&](StageVec<PX> (&sv)[8], int ch0) {
        const unsigned sbase = (unsigned)ch0 * st.cstride;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const unsigned vo = (st.cfull || ch0 + st.hu8 + j < st.C) ? st.voff : ffc::OOB;
            sv[j] = stage_ld<PX>(st.rs, (int)vo, (int)(sbase + (unsigned)j * st.cstride));
        }
    };
    auto stage_store = [&](const StageVec<PX> (&sv)[8], int wb, char* buf) {
        if (wb >= 0) {
#pragma unroll
            for (int e = 0; e < PX; ++e) {
                float v8[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) v8[j] = sv[j].v[e];
                const Split3 sp = split3(v8);
                u32x4* d = reinterpret_cast<u32x4*>(buf + wb + 48 * e);
                d[0] = __builtin_bit_cast(u32x4, sp.hi);
                d[1] = __builtin_bit_cast(u32x4, sp.mid);
                d[2] = __builtin_bit_cast(u32x4, sp.lo);
            }
        }
    };

    // per-segment compute geometry: LDS byte offset of the lane's B fragment per (N-tile, tap);
    // staged segments always run 4 taps (the plan pads missing ones with zero weights)
    int kseg = 0, cpad = 0;
    int fb[NTW];        // per N-tile: byte offset of (h, lane pixel) inside a buffer
    int tb[4];          // per tap: byte offset of the tap's pixel shift
    auto geom = [&](int s, int (&fbo)[NTW], int (&tbo)[4]) {
        const ffc_convp_seg& S = J.seg[s];
        const QGeom<NTW> g = q_geometry<NTW>(J, wave, lane, pb);
        const int QR = S.qrow, QS = S.qsample, nimg = NS * QS;
        const int ix0 = c0 * S.mult_x + S.org_x, xoff = ix0 - (ix0 & ~3);
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt)
            fbo[nt] = (h * nimg + g.pns[nt] * QS + g.pr_[nt] * S.mult_y * QR + g.pc_[nt] * S.mult_x + xoff) * 48;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int tt = P.tap[s][t];
            tbo[t] = ((tt >> 16) * QR + (tt & 0xFFFF)) * 48;
        }
    };
    auto compute_setup = [&](int s) {
        kseg = P.kseg[s];
        cpad = J.seg[s].Cpad;
        geom(s, fb, tb);
    };

    // K = the staged segments' 16-channel chunks (in job order), then the direct segments' chunks;
    // K split ks of nsplit takes the chunk range [lo, hi) of that sequence
    int nstaged = 0, ndirect = 0;
    for (int s = 0; s < nseg; ++s) {
        if (J.seg[s].direct) ndirect += J.seg[s].Cpad >> 4;
        else nstaged += J.seg[s].Cpad >> 4;
    }
    const int ntot = nstaged + ndirect;
    const int lo = ntot * ks / nsplit, hi = ntot * (ks + 1) / nsplit;
    const int slo = min(lo, nstaged), nst = min(hi, nstaged) - slo;
    const int dlo = max(lo, nstaged) - nstaged, dhi = max(hi, nstaged) - nstaged;

    const int npad = (nst + SL - 1) / SL * SL;   // barrier periods after the first (>= nst)
    if (nst > 0) {
        int ss = 0;
        while (J.seg[ss].direct) ++ss;
        int c0k = slo;   // first chunk of this split: segment ss, chunk c0k inside it
        while (c0k >= (J.seg[ss].Cpad >> 4)) {
            c0k -= J.seg[ss].Cpad >> 4;
            do { ++ss; } while (J.seg[ss].direct);
        }
        int cs = ss, sch = 16 * c0k, cch = 16 * c0k;   // stager / computer: segment and channel of their chunk
        // Three LDS buffers: chunk k is stored into buffer k % 3 two barrier periods before the compute
        // waves finish chunk k - 1, so during chunk k - 1 both buffers k - 1 and k are complete and the
        // compute waves read chunk k's first tap before the barrier (its LDS latency then sits under
        // the last tap's MFMAs instead of at the head of every chunk).  Barrier B0 follows the
        // staging of chunks 0 and 1; period c (1 .. npad) stores chunk c + 1 and ends with barrier Bc;
        // the compute waves run chunk ci between B(ci) and B(ci + 1).
        if (stager) {
#ifdef FFC_TRACE_Q
            unsigned long long q0, qa, qb, ql = 0, qs = 0, qw = 0, qi = 0;
            QSTAMP(q0);
#endif
            StageVec<PX> sv[SL][8];
            int wbs[SL];
            stage_setup(ss);
            // the chunk at the load cursor (ss, sch); past the last chunk the loads still issue (the
            // previous addresses, no store): every period then has the same load / wait pattern, so
            // the compiler's wait counts stay exact (a conditional issue made it wait for every
            // outstanding load at the loop head, serialising the pipeline)
            int ic = 0;   // chunks issued (this workgroup's K range is chunks 0 .. nst - 1)
            auto issue = [&](StageVec<PX> (&dst)[8], int& wb) {
                const bool live = ss < nseg && ic < nst;
                ++ic;
                stage_load(dst, live ? sch : 0);
                wb = live ? st.wb : -1;
                if (live) {
                    sch += 16;
                    if (sch >= st.Cpad) {   // next staged segment (kernel-argument loads only here)
                        do { ++ss; } while (ss < nseg && J.seg[ss].direct);
                        sch = 0;
                        if (ss < nseg) stage_setup(ss);
                    }
                }
            };
            auto store_timed = [&](const StageVec<PX> (&src)[8], int wb, char* buf) {
#ifdef FFC_TRACE_Q
                QSTAMP(qa);
                float chk = src[0].v[0] + src[7].v[PX - 1];
                asm volatile("" ::"v"(chk));   // data arrived
                QSTAMP(qb);
                ql += qb - qa;
                stage_store(src, wb, buf);
                QSTAMP(qa);
                qs += qa - qb;
#else
                stage_store(src, wb, buf);
#endif
            };
            auto bar = [&]() {
#ifdef FFC_TRACE_Q
                QSTAMP(qa);
#endif
#ifndef FFC_QPROBE_NOBAR
                __syncthreads();   // chunk c + 1 written; everyone done reading chunk c - 1's buffer
#endif
#ifdef FFC_TRACE_Q
                QSTAMP(qb);
                qw += qb - qa;
#endif
            };
            // SL register slots (chunk k in slot k % SL; the loop is unrolled by SL so
            // every slot index is a compile-time constant): the loads of chunks c + 2 .. c + SL are
            // in flight while chunk c + 1 is split and stored
#pragma unroll
            for (int u = 0; u < SL; ++u) issue(sv[u], wbs[u]);
            store_timed(sv[0], wbs[0], lds);
            issue(sv[0], wbs[0]);                                   // chunk SL
            store_timed(sv[1 % SL], wbs[1 % SL], lds + ebuf);
            bar();   // B0
            int wbuf = 2;   // buffer of the chunk stored next (chunk c + 1 of period c)
            // periods 1 .. npad (nst rounded up to whole SL-period rounds: no exit in the middle of the
            // unrolled body, so every path into the loop head has the same loads in flight); periods
            // past the last chunk issue nothing live, store nothing and only meet the compute waves'
            // barriers
            for (int c0 = 1; c0 <= npad; c0 += SL) {
#pragma unroll
                for (int u = 0; u < SL; ++u) {   // period c = c0 + u: c % SL == (1 + u) % SL
#ifndef FFC_QPROBE_NOSTAGE
#ifdef FFC_TRACE_Q
                    QSTAMP(qa);
#endif
                    issue(sv[(1 + u) % SL], wbs[(1 + u) % SL]);   // chunk c + SL
#ifdef FFC_TRACE_Q
                    QSTAMP(qb);
                    qi += qb - qa;
#endif
                    store_timed(sv[(2 + u) % SL], wbs[(2 + u) % SL], lds + wbuf * ebuf);   // chunk c + 1
#endif
                    wbuf = wbuf == 2 ? 0 : wbuf + 1;
                    bar();
                }
            }
#ifdef FFC_TRACE_Q
            QSTAMP(qa);
            if (tid == 256) {
                unsigned long long* tr = g_ffc_trace_q + 16 * tix;
                tr[9] = ql;
                tr[10] = qs;
                tr[11] = qw;
                tr[12] = qa - q0;
                tr[13] = nst;
                tr[14] = qi;
            }
#endif
            return;   // no barrier follows
        }
        // A of the current chunk, refilled tap by tap with the next chunk's right after the tap's
        // MFMAs: every A load has a whole chunk of MFMAs to arrive in (L2 latency under load is
        // ~1-2K cycles; loading taps 1-3 at the chunk start exposed it), in the same registers
        Split3 a[4][MT];
        compute_setup(cs);
        int pf[NTW];   // byte offsets of the next chunk's tap-0 fragments (its segment's geometry)
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) pf[nt] = fb[nt] + tb[0];
#pragma unroll
        for (int t = 0; t < 4; ++t) load_A(kseg + cch * 4 + 16 * t, a[t]);
        // B fragments of a whole tap (NTW x 3 ds_read_b128) one tap ahead of its MFMAs
        u32x4 bq[2][NTW][3];
        auto read_frag = [&](const char* base, const int (&off)[NTW], int add, u32x4 (&dst)[NTW][3]) {
#pragma unroll
            for (int nt = 0; nt < NTW; ++nt) {
                const char* p1 = base + off[nt] + add;
                dst[nt][0] = lds_read16(p1, 0);
                dst[nt][1] = lds_read16(p1, 16);
                dst[nt][2] = lds_read16(p1, 32);
            }
        };
#ifdef FFC_TRACE_Q
        QSTAMP(tq_a);
#endif
        __syncthreads();   // B0: chunks 0 and 1 stored
#ifdef FFC_TRACE_Q
        QSTAMP(tq_b);
        tq_bar += tq_b - tq_a;
#endif
        read_frag(lds, pf, 0, bq[0]);   // chunk 0, tap 0
        int rbuf = 0;
        for (int ci = 0; ci < nst; ++ci) {
#ifdef FFC_TRACE_Q
            QSTAMP(tq_a);
#endif
            const bool more = ci + 1 < nst;
            const int nbuf = rbuf == 2 ? 0 : rbuf + 1;
            const char* cur = lds + rbuf * ebuf;
            const char* nxt = lds + nbuf * ebuf;
            // the next chunk (segment cn, channel chn): its K base for the A refill and, on a segment
            // change, its tap-0 fragment offsets for the prefetch (kernel-argument loads only then)
            int cn = cs, chn = cch + 16;
            const bool segchg = more && chn >= cpad;
            int kn;
            if (segchg) {
                do { ++cn; } while (J.seg[cn].direct);
                chn = 0;
                kn = P.kseg[cn];
                int fbn[NTW], tbn[4];
                geom(cn, fbn, tbn);
#pragma unroll
                for (int nt = 0; nt < NTW; ++nt) pf[nt] = fbn[nt] + tbn[0];
            } else {
                // the last chunk reloads its own A: no branch around the loads
                kn = kseg + (more ? chn : cch) * 4;
            }
            __builtin_amdgcn_sched_barrier(0);
#ifdef FFC_TRACE_Q
            QSTAMP(tq_b);
            tq_A += tq_b - tq_a;
#endif
#ifndef FFC_QPROBE_NOMFMA
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                // tap t + 1's fragments, or the next chunk's tap 0 (read from the other complete
                // buffer; past the last chunk a harmless read of data nobody uses)
                if (t + 1 < 4) read_frag(cur, fb, tb[t + 1], bq[(t + 1) & 1]);
                else read_frag(nxt, pf, 0, bq[0]);
#pragma unroll
                for (int nt = 0; nt < NTW; ++nt) {
                    Split3 b;
                    b.hi = __builtin_bit_cast(bf16x8, bq[t & 1][nt][0]);
                    b.mid = __builtin_bit_cast(bf16x8, bq[t & 1][nt][1]);
                    b.lo = __builtin_bit_cast(bf16x8, bq[t & 1][nt][2]);
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt) acc[mt][nt] = mfma_split3(a[t][mt], b, acc[mt][nt]);
                }
#ifndef FFC_QPROBE_NOA   // timing probe only: A of the first chunk reused
                load_A(kn + 16 * t, a[t]);   // refill: the next chunk's tap t
#endif
                // keep the next reads ahead of this tap's MFMAs (the scheduler otherwise sinks each
                // read to just before its first use and waits on it), the refill after them
                __builtin_amdgcn_sched_group_barrier(0x100, 3 * NTW, 0);   // DS_READ
                __builtin_amdgcn_sched_group_barrier(0x8, 6 * NTW * MT, 0);  // MFMA
                __builtin_amdgcn_sched_group_barrier(0x20, 3 * MT, 0);       // VMEM_READ
                __builtin_amdgcn_sched_barrier(0);
            }
#endif
#ifdef FFC_TRACE_Q
            QSTAMP(tq_a);
            tq_mf += tq_a - tq_b;
#endif
            if (segchg) {
                cs = cn;
                cch = 0;
                compute_setup(cs);
            } else {
                cch += 16;
            }
            rbuf = nbuf;
#ifdef FFC_TRACE_Q
            QSTAMP(tq_a);
#endif
#ifndef FFC_QPROBE_NOBAR
            __syncthreads();   // chunk ci + 2 written; everyone done reading chunk ci
#endif
#ifdef FFC_TRACE_Q
            QSTAMP(tq_b);
            tq_bar += tq_b - tq_a;
#endif
        }
#ifndef FFC_QPROBE_NOBAR
        for (int ci = nst; ci < npad; ++ci) __syncthreads();   // the staging waves' padding periods
#endif
    }
#ifdef FFC_TRACE_Q
    QSTAMP(tq_c);
#endif
    if (stager) return;   // no barrier follows

    // ---------------- direct segments (1x1 at the output resolution): B straight from global
    int dbase = 0;
    for (int s = 0; s < nseg; ++s) {
        const ffc_convp_seg& S = J.seg[s];
        if (!S.direct) continue;
        const int nch = S.Cpad >> 4;
        const int c_lo = max(dlo - dbase, 0), c_hi = min(dhi - dbase, nch);
        dbase += nch;
        if (c_lo >= c_hi) continue;
        const int IHW = S.IH * S.IW;
        const QGeom<NTW> g = q_geometry<NTW>(J, wave, lane, pb);
        const bool* pv = g.pv;
        const float* xp[NTW];
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) {
            const int oy = (r0 + g.pr_[nt]) * J.Sy + P.py, ox = (c0 + g.pc_[nt]) * J.Sx + P.px;
            const int b = pv[nt] ? b0 + g.pns[nt] : 0;
            xp[nt] = S.x + ((long long)b * S.C + 8 * h) * IHW + (pv[nt] ? oy * S.IW + ox : 0);
        }
        for (int ch0 = 16 * c_lo; ch0 < 16 * c_hi; ch0 += 16) {
            Split3 a[MT];
            load_A(P.kseg[s] + ch0, a);
            float bv[NTW][8];
#pragma unroll
            for (int nt = 0; nt < NTW; ++nt)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const bool ok = pv[nt] && ch0 + 8 * h + j < S.C;
                    const float v = (ok ? xp[nt] : S.x)[ok ? (long long)(ch0 + j) * IHW : 0];
                    bv[nt][j] = ok ? v : 0.0f;
                }
#pragma unroll
            for (int nt = 0; nt < NTW; ++nt) {
                const Split3 b = split3(bv[nt]);
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) acc[mt][nt] = mfma_split3(a[mt], b, acc[mt][nt]);
            }
        }
    }

#ifdef FFC_QPROBE_NOEPI
    if (acc[0][0][0] != 1234.5f) return;   // keep the accumulators live, skip the stores
#endif
    // ---------------- K split: store this split's fragments; convq_reduce_kernel adds them
    if (nsplit > 1) {
        store_partial<MT, NTW>(args.part + ((size_t)(slot * nsplit + ks) * 4 + wave) * (MT * NTW * 1024), lane, acc);
        return;
    }
#ifdef FFC_TRACE_Q
    QSTAMP(tq_d);
#endif
    convq_epilogue<MT, NTW>(J, wave, lane, pb, m0, acc);
#ifdef FFC_TRACE_Q
    {
        unsigned long long tq_e;
        QSTAMP(tq_e);
        if (tid == 0) {
            unsigned long long* tr = g_ffc_trace_q + 16 * tix;
            tr[0] = tq_rt0;
            tr[1] = __builtin_amdgcn_s_memrealtime();
            tr[2] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                    ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);
            tr[3] = tq_bar;
            tr[4] = tq_A;
            tr[5] = tq_mf;
            tr[6] = tq_d - tq_c;
            tr[7] = tq_e - tq_d;
            tr[8] = tq_e - tq_0;
        }
    }
#endif
}

// Persistent over the tile table: workgroup b runs tiles b, b + G, b + 2G, ... (G = gridDim.x, a
// multiple of 8, so every tile of a workgroup comes from its XCD's range of the XCD-remapped table).
// A tile's epilogue stores drain while the staging waves already load and split the next tile's
// first chunk, and the next tile's MFMAs start without a fresh workgroup launch.
template <int MT, int NTW, int SL = QSLOTS, int PX = 4>
__global__ __launch_bounds__(QTHREADS) FFC_CONVQ_WPE void convq_kernel(ConvQArgs args_byval) {
#if defined(__HIP_DEVICE_COMPILE__)
    const ConvQArgs& args = *(const ConvQArgs*)__builtin_amdgcn_kernarg_segment_ptr();
#else
    const ConvQArgs& args = args_byval;
#endif
    extern __shared__ __attribute__((aligned(16))) char lds[];
    for (int tix = blockIdx.x; tix < args.ntiles; tix += gridDim.x) convq_tile<MT, NTW, SL, PX>(args, tix, lds);
}

// K split, second pass: workgroup = one output tile (slot), wave w = phase w; adds the ksplit
// partial fragments in split order (deterministic) and runs the epilogue.  A separate launch
// rather than a last-arriver in convq_kernel: making the partials visible across XCDs from inside
// the kernel takes an L2 writeback per wave (buffer_wbl2), which cost more than the split saved.
template <int MT, int NTW>
__global__ __launch_bounds__(256) void convq_reduce_kernel(ConvQArgs args_byval, const int4* __restrict__ slots) {
#if defined(__HIP_DEVICE_COMPILE__)
    const ConvQArgs& args = *(const ConvQArgs*)__builtin_amdgcn_kernarg_segment_ptr();
#else
    const ConvQArgs& args = args_byval;
#endif
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int4 tile = slots[blockIdx.x];
    const int ji = __builtin_amdgcn_readfirstlane(tile.x);
    const int m0 = __builtin_amdgcn_readfirstlane(tile.y);
    const int pb = __builtin_amdgcn_readfirstlane(tile.z);
    const int nsplit = args.ksplit;
    constexpr int FR = MT * NTW * 1024;
    const float* base = args.part + ((size_t)blockIdx.x * nsplit * 4 + wave) * FR + lane * 4;
    floatx16 acc[MT][NTW];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt)
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4) {
                // all nsplit (<= 8) partials in flight at once: clamped loads, then the sum in split order
                const float* p = base + ((mt * NTW + nt) * 4 + r4) * 256;
                floatx4 v[8];
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    v[k] = *reinterpret_cast<const floatx4*>(p + (size_t)(k < nsplit ? k : 0) * 4 * FR);
                floatx4 sum = v[0];
#pragma unroll
                for (int k = 1; k < 8; ++k)
                    if (k < nsplit) sum += v[k];
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[mt][nt][4 * r4 + e] = sum[e];
            }
    convq_epilogue<MT, NTW>(args.jobs[ji], wave, lane, pb, m0, acc);
}

// Workgroups of the persistent grid: every CU's resident workgroups (occupancy of this kernel at this
// LDS size, queried once per (kernel, LDS bytes, device)), rounded down to a multiple of 8 (the XCD
// count: workgroup b then stays on XCD b % 8 for all its tiles), never more than the tiles.
// FFC_CONVQ_PERSIST=0 launches one workgroup per tile (the previous grid; A/B measurements).
int persistent_grid(const void* k, size_t lds, int ntiles) {
    static const bool off = [] {
        const char* e = getenv("FFC_CONVQ_PERSIST");
        return e && e[0] == '0';
    }();
    if (off) return ntiles;
    static std::mutex mu;
    static std::map<std::tuple<const void*, size_t, int>, int> cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        ffc::set_error("ffc_convq_forward: hipGetDevice failed");
        return -1;
    }
    int slots = 0;
    {
        std::lock_guard<std::mutex> g(mu);
        auto it = cache.find({k, lds, dev});
        if (it != cache.end()) {
            slots = it->second;
        } else {
            int cus = 0, per = 0;
            if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
                hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, QTHREADS, lds) != hipSuccess || cus <= 0) {
                ffc::set_error("ffc_convq_forward: occupancy query failed");
                return -1;
            }
            slots = cus * (per > 0 ? per : 1);
            slots = slots >= 8 ? slots / 8 * 8 : slots;
            cache[{k, lds, dev}] = slots;
        }
    }
    return ntiles < slots ? ntiles : slots;
}

template <int MT, int NTW, int SL = QSLOTS, int PX = 4>
int launch_q(const ConvQArgs& a, int ntiles, size_t lds, hipStream_t s, const int4* slots, int nslots) {
    auto k = convq_kernel<MT, NTW, SL, PX>;
    if (lds > 64 * 1024) {
        static bool raised = false;   // per instantiation
        if (!raised) {
            const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            if (e != hipSuccess) {
                ffc::set_error(std::string("ffc_convq_forward: hipFuncSetAttribute: ") + hipGetErrorString(e));
                return FFC_E_LAUNCH;
            }
            raised = true;
        }
    }
    const int grid = persistent_grid(reinterpret_cast<const void*>(k), lds, ntiles);
    if (grid <= 0) return FFC_E_LAUNCH;
    hipLaunchKernelGGL(k, dim3(grid), dim3(QTHREADS), lds, s, a);
    if (a.ksplit > 1) {
        const int rc = ffc::launch_status("ffc_convq_forward_split");
        if (rc != FFC_OK) return rc;
        auto r = convq_reduce_kernel<MT, NTW>;
        hipLaunchKernelGGL(r, dim3(nslots), dim3(256), 0, s, a, slots);
    }
    return ffc::launch_status("ffc_convq_forward_split");
}

int stage_px(int units4) {
    static const int force = [] {
        const char* e = getenv("FFC_CONVQ_PX");
        return e ? atoi(e) : 0;
    }();
    const int fit = 4 * units4 <= 256 ? 1 : (2 * units4 <= 256 ? 2 : 4);   // one unit per staging thread
    return (force == 1 || force == 2 || force == 4) && force >= fit ? force : fit;
}

int slots11() {
    static const int v = [] {
        const char* e = getenv("FFC_CONVQ_SLOTS11");
        const int n = e ? atoi(e) : 0;
        return (n == 3 || n == 4) ? n : QSLOTS;
    }();
    return v;
}

}  // namespace

namespace {
// the transcendental activations of a convq job's output, in place (see q_slope)
__global__ void q_act_inplace_kernel(float* __restrict__ x, long long n, int act) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const float v = x[i];
        float y;
        switch (act) {
            case FFC_ACT_TANH: y = tanhf(v); break;
            case FFC_ACT_SIGMOID: y = 1.0f / (1.0f + expf(-v)); break;
            default: y = 0.5f * v * (1.0f + erff(v * 0.70710678118654752f)); break;   // FFC_ACT_GELU
        }
        x[i] = y;
    }
}

// A[phase][Mpad][Kpad] fp32 -> fragment-ordered split planes: element
// 3 * a_off + ((mtile * Kpad/16 + kstep) * 3 + piece) * 512 + lane * 8 + j  holds piece `piece` of
// A[m = 32 * mtile + (lane & 31)][k = 16 * kstep + 8 * (lane >> 5) + j]
__global__ void pack_a3_kernel(const float* __restrict__ A, ffc_convp_job J, uint16_t* __restrict__ A3, long long total) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
        // i = (phase-local fragment lane) over all phases: find the phase
        long long r = i;
        int p = 0;
        long long nfr = 0;
        for (; p < J.nphase; ++p) {
            nfr = (long long)(J.Mpad >> 5) * (J.ph[p].Kpad >> 4) * 64;
            if (r < nfr) break;
            r -= nfr;
        }
        const int lane = (int)(r & 63);
        const long long fr = r >> 6;
        const int ks = J.ph[p].Kpad >> 4;
        const int mtile = (int)(fr / ks), kstep = (int)(fr - (long long)mtile * ks);
        const int m = 32 * mtile + (lane & 31), k0 = 16 * kstep + 8 * (lane >> 5);
        const float* src = A + J.ph[p].a_off + (size_t)m * J.ph[p].Kpad + k0;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = src[j];
        const Split3 sp = split3(v);
        uint16_t* dst = A3 + 3 * J.ph[p].a_off + (fr * 3) * 512 + lane * 8;
        *reinterpret_cast<u32x4*>(dst) = __builtin_bit_cast(u32x4, sp.hi);
        *reinterpret_cast<u32x4*>(dst + 512) = __builtin_bit_cast(u32x4, sp.mid);
        *reinterpret_cast<u32x4*>(dst + 1024) = __builtin_bit_cast(u32x4, sp.lo);
    }
}
}  // namespace

extern "C" int ffc_convq_pack_a3(const ffc_convp_job* job, const float* A, uint16_t* A3, void* stream) {
    FFC_CHECK_ARG(job && A && A3 && job->nphase >= 1 && job->nphase <= 4 && job->Mpad % 32 == 0,
                  "ffc_convq_pack_a3: bad args");
    FFC_CHECK_ARG((reinterpret_cast<uintptr_t>(A3) & 15) == 0, "ffc_convq_pack_a3: A3 must be 16-byte aligned");
    long long total = 0;
    for (int p = 0; p < job->nphase; ++p) {
        FFC_CHECK_ARG(job->ph[p].Kpad % 16 == 0 && job->ph[p].Kpad > 0, "ffc_convq_pack_a3: Kpad % 16");
        total += (long long)(job->Mpad >> 5) * (job->ph[p].Kpad >> 4) * 64;
    }
    const long long blocks = (total + 255) / 256;
    hipLaunchKernelGGL(pack_a3_kernel, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(256), 0,
                       (hipStream_t)stream, A, *job, A3, total);
    return ffc::launch_status("ffc_convq_pack_a3");
}

#ifdef FFC_TRACE_Q
extern "C" int ffc_debug_trace_read_q(void* dst, size_t bytes) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_ffc_trace_q), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int ffc_convq_config(int cfg, int* mt, int* ntw) {
    static const int T[4][2] = {{1, 4}, {1, 2}, {2, 2}, {1, 1}};
    if (cfg < 0 || cfg > 3 || !mt || !ntw) return FFC_E_INVALID;
    *mt = T[cfg][0];
    *ntw = T[cfg][1];
    return FFC_OK;
}

extern "C" long long ffc_convq_split_floats(int cfg, int nslots, int ksplit) {
    int MT = 0, NTW = 0;
    if (ffc_convq_config(cfg, &MT, &NTW) != FFC_OK || nslots < 0 || ksplit < 1 || ksplit > 8) return -1;
    return ksplit > 1 ? (long long)nslots * ksplit * 4 * MT * NTW * 1024 : 0;
}

extern "C" int ffc_convq_forward(const ffc_convp_job* jobs, int njobs, const int* tiles, int ntiles, int cfg,
                                 void* stream) {
    return ffc_convq_forward_split(jobs, njobs, tiles, ntiles, nullptr, 0, cfg, 1, nullptr, stream);
}

extern "C" int ffc_convq_forward_split(const ffc_convp_job* jobs, int njobs, const int* tiles, int ntiles,
                                       const int* slot_tiles, int nslots, int cfg, int ksplit, float* part,
                                       void* stream) {
    FFC_CHECK_ARG(jobs && tiles && njobs >= 1 && njobs <= 2 && ntiles > 0, "ffc_convq_forward: bad args");
    int MT = 0, NTW = 0;
    FFC_CHECK_ARG(ffc_convq_config(cfg, &MT, &NTW) == FFC_OK, "ffc_convq_forward: unknown cfg");
    FFC_CHECK_ARG(ksplit >= 1 && ksplit <= 8, "ffc_convq_forward: 1 <= ksplit <= 8");
    FFC_CHECK_ARG(ksplit == 1 || (part && (reinterpret_cast<uintptr_t>(part) & 15) == 0),
                  "ffc_convq_forward: ksplit > 1 needs the partial buffer (16-byte aligned)");
    FFC_CHECK_ARG(ksplit == 1 || (slot_tiles && nslots > 0 && (long long)nslots * ksplit == ntiles),
                  "ffc_convq_forward: ksplit > 1 needs the slot table (ntiles = nslots * ksplit)");
    int npix_max = 0, units4 = 0;
    for (int j = 0; j < njobs; ++j) {
        const ffc_convp_job& J = jobs[j];
        FFC_CHECK_ARG(J.A3 && J.out && J.B > 0 && J.M > 0, "ffc_convq_forward: incomplete job (needs the A3 planes)");
        FFC_CHECK_ARG((reinterpret_cast<uintptr_t>(J.A3) & 15) == 0 && J.a3_stride % 8 == 0,
                      "ffc_convq_forward: A3 planes need 16-byte alignment");
        FFC_CHECK_ARG(J.nphase == 4 && J.Sy == 2 && J.Sx == 2, "ffc_convq_forward: 4-phase (stride-2) jobs only");
        FFC_CHECK_ARG(J.nseg >= 1 && J.nseg <= FFC_MAX_SEG, "ffc_convq_forward: nseg out of range");
        FFC_CHECK_ARG(J.Mpad % 128 == 0 && J.Mpad >= J.M, "ffc_convq_forward: Mpad");
        FFC_CHECK_ARG((unsigned long long)J.NS * J.M * J.OH * J.OW * 4 < 0xFFFFFFFFull,
                      "ffc_convq_forward: a pixel block's output span must fit 32-bit offsets");
        FFC_CHECK_ARG(J.NS > 0 && J.TR > 0 && J.TC > 0 && J.nrb > 0 && J.ncb > 0 && J.NS * J.TR * J.TC <= 32 * NTW,
                      "ffc_convq_forward: pixel block");
        for (int p = 0; p < 4; ++p) FFC_CHECK_ARG(J.ph[p].Kpad % 16 == 0, "ffc_convq_forward: Kpad % 16");
        for (int s = 0; s < J.nseg; ++s) {
            const ffc_convp_seg& S = J.seg[s];
            FFC_CHECK_ARG(S.x && S.Cpad % 16 == 0 && S.Cpad >= S.C && S.cc == 16, "ffc_convq_forward: segment channels");
            FFC_CHECK_ARG(!S.pool && !S.gate, "ffc_convq_forward: pooled / gated segments use ffc_conv_forward");
            for (int p = 0; p < 4; ++p) {
                const int T = J.ph[p].T[s];
                FFC_CHECK_ARG(S.direct ? T == 1 : T == 4,
                              "ffc_convq_forward: taps per phase (4 staged, 1 direct; the plan pads)");
            }
            if (S.direct) {
                FFC_CHECK_ARG(S.mult_y == 2 && S.mult_x == 2 && S.IH == J.OH && S.IW == J.OW,
                              "ffc_convq_forward: direct segments are 1x1 at the output resolution");
            } else {
                FFC_CHECK_ARG(S.PR > 0 && S.PC > 0 && S.PC % 4 == 0 && S.qrow >= S.PC && S.qsample >= S.PR * S.qrow,
                              "ffc_convq_forward: patch shape / LDS strides");
                FFC_CHECK_ARG(S.vec4 && S.IW % 4 == 0 && (reinterpret_cast<uintptr_t>(S.x) & 15) == 0,
                              "ffc_convq_forward: staged segments need IW % 4 == 0 and a 16-byte aligned input");
                FFC_CHECK_ARG((unsigned long long)J.B * S.C * S.IH * S.IW * 4 < 0x7FFFFFFFull,
                              "ffc_convq_forward: staged segments are read through 32-bit buffer offsets (< 2 GiB)");
                FFC_CHECK_ARG(2 * J.NS * S.PR * (S.PC / 4) <= 256,
                              "ffc_convq_forward: patch too large for the staging waves (one unit per thread)");
                if (2 * J.NS * S.PR * (S.PC / 4) > units4) units4 = 2 * J.NS * S.PR * (S.PC / 4);
                const int npix = J.NS * S.qsample;   // LDS image pixels per channel half
                if (npix > npix_max) npix_max = npix;
            }
        }
    }
    const size_t ebuf = ((size_t)npix_max * 96 + 255) / 256 * 256 + 256;   // + 256 B: buffers start on other banks
    size_t lds = npix_max > 0 ? 3 * ebuf : 16;   // three chunk buffers (convq_tile)
    FFC_CHECK_ARG(lds <= 160 * 1024, "ffc_convq_forward: patch too large");
    ConvQArgs a;
    a.ebuf = (int)ebuf;
    a.jobs[0] = jobs[0];
    a.jobs[1] = jobs[njobs > 1 ? 1 : 0];
    a.tiles = reinterpret_cast<const int4*>(tiles);
    a.ksplit = ksplit;
    a.part = part;
    a.ntiles = ntiles;
    const int4* sl = reinterpret_cast<const int4*>(slot_tiles);
    hipStream_t s = (hipStream_t)stream;
    // Tanh / Sigmoid / GELU: the kernel stores the pre-activation, a second pass applies it (q_slope)
    bool post[2] = {false, false};
    for (int j = 0; j < 2; ++j) {
        ffc_convp_job& Jc = a.jobs[j];
        if (Jc.act == FFC_ACT_TANH || Jc.act == FFC_ACT_SIGMOID || Jc.act == FFC_ACT_GELU) {
            post[j] = j < njobs;
            Jc.act = FFC_ACT_IDENTITY;
        }
    }
    // pixels per staging unit: the smallest of 1, 2, 4 whose units fit the 256 staging threads
    // (FFC_CONVQ_PX = 4 keeps the 4-pixel units everywhere: A/B; the (1, 4) and (2, 2) tiles with
    // 2-pixel units measured neutral on gen64 and 0.3-1 % faster on fgan128's conv, r05y / r05aa)
    const int px = stage_px(units4);
    int rc = FFC_E_INVALID;
    switch (cfg) {
        case 0:
            if (px <= 2) rc = launch_q<1, 4, QSLOTS, 2>(a, ntiles, lds, s, sl, nslots);
            else rc = launch_q<1, 4>(a, ntiles, lds, s, sl, nslots);
            break;
        case 1:
            if (px <= 2) rc = launch_q<1, 2, QSLOTS, 2>(a, ntiles, lds, s, sl, nslots);
            else rc = launch_q<1, 2>(a, ntiles, lds, s, sl, nslots);
            break;
        case 2:
            if (px <= 2) rc = launch_q<2, 2, QSLOTS, 2>(a, ntiles, lds, s, sl, nslots);
            else rc = launch_q<2, 2>(a, ntiles, lds, s, sl, nslots);
            break;
        case 3:
            // the (1, 1) tile: pixels per staging unit by the patch size (stage_px); FFC_CONVQ_SLOTS11 = 3 | 4
            // keeps more chunks' loads in flight (measured slower: it halves the workgroups per CU, r05a)
            if (slots11() == 3) rc = launch_q<1, 1, 3>(a, ntiles, lds, s, sl, nslots);
            else if (slots11() == 4) rc = launch_q<1, 1, 4>(a, ntiles, lds, s, sl, nslots);
            else if (px == 1) rc = launch_q<1, 1, QSLOTS, 1>(a, ntiles, lds, s, sl, nslots);
            else if (px == 2) rc = launch_q<1, 1, QSLOTS, 2>(a, ntiles, lds, s, sl, nslots);
            else rc = launch_q<1, 1>(a, ntiles, lds, s, sl, nslots);
            break;
        default: ffc::set_error("ffc_convq_forward: unknown cfg"); return FFC_E_INVALID;
    }
    if (rc != FFC_OK) return rc;
    for (int j = 0; j < njobs; ++j) {
        if (!post[j]) continue;
        const long long n = (long long)jobs[j].B * jobs[j].M * jobs[j].OH * jobs[j].OW;
        const long long blocks = (n + 255) / 256;
        hipLaunchKernelGGL(q_act_inplace_kernel, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256), 0, s,
                           jobs[j].out, n, jobs[j].act);
        rc = ffc::launch_status("ffc_convq_forward (activation pass)");
        if (rc != FFC_OK) return rc;
    }
    return FFC_OK;
}
