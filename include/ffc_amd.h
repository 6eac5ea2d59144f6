/*
 * ffc_amd.h — C ABI of the MI355X-native Fast Fourier Convolution hot path.
 *
 * The reference (phbgomes22/FastFourierConvolution) is pure PyTorch: its hot path
 * (BASELINE.json north_star) is the layers/ffc operator surface whose arithmetic
 * runs inside ATen.  It has no FFI of its own; the entry points below are what a
 * binding for that surface needs, and each names the reference interface it
 * replaces.  Every entry point:
 *   - takes plain device pointers, sizes and a hipStream_t (passed as void*),
 *   - launches asynchronously on that stream only (no allocation, no host sync,
 *     so callers may capture it into a hipGraph),
 *   - returns 0 on success or a negative FFC_E_* code; ffc_last_error() then
 *     returns a thread-local message.
 * All tensors are fp32, NCHW, contiguous.  PyTorch owns every buffer.
 */
#ifndef FFC_AMD_H
#define FFC_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FFC_OK 0
#define FFC_E_INVALID (-1)     /* bad argument / unsupported shape */
#define FFC_E_LAUNCH (-2)      /* hipLaunchKernel failed */

#define FFC_MAX_SEG 3
#define FFC_MAX_PHASE 16

/* activation codes (layers/ffc/ffc_bn_act.py:63-67; LeakyReLU slope 0.1 passed in act_param) */
#define FFC_ACT_IDENTITY 0
#define FFC_ACT_RELU 1
#define FFC_ACT_LEAKY_RELU 2
#define FFC_ACT_TANH 3
#define FFC_ACT_SIGMOID 4
#define FFC_ACT_GELU 5

const char* ffc_last_error(void);
int ffc_abi_version(void);
/* sizeof(ffc_conv_seg), (ffc_conv_phase), (ffc_conv_job), (ffc_convp_seg), (ffc_convp_phase),
 * (ffc_convp_job) -> out[0..5]; n >= 7: sizeof(ffc_bn_fold) -> out[6]; n >= 8: sizeof(ffc_in_tf) -> out[7];
 * n >= 10: sizeof(ffc_bn_rf_item), sizeof(ffc_bn_apply_item) -> out[8], out[9] */
int ffc_struct_sizes(int* out, int n);

/* ------------------------------------------------------------------ local branch
 * Implicit-GEMM convolution / transposed convolution with several input segments
 * summed into one output (FFC.forward's convl2l(x_l)+convg2l(x_g),
 * layers/ffc/ffc.py:89-97; FFCTranspose.forward, layers/ffc/ffc_transpose.py:96-106;
 * and SpectralTransform's 1x1 conv1 / conv2, layers/ffc/spectral_transform.py:89,108).
 * Output pixels are split into phases (oy = my*Sy + py); within a phase the taps are
 * uniform, so each phase is one GEMM  out[m, n] = sum_k A[phase][m][k] * B(k, n),
 * B gathered on the fly from the segments through the per-phase k-table.
 */
typedef struct ffc_conv_seg {
    const float* x;      /* (B, C, IH, IW) or (B, C, 2IH, 2IW) when pool=1 */
    const float* gate;   /* optional (B, C) multiplier (SE gate), or NULL */
    int C, IH, IW;       /* logical input dims seen by the taps */
    int mult_y, mult_x;  /* input coord = m*mult + off */
    int pool;            /* 1: 2x2 average pool applied on the fly (AvgPool2d(2,2)) */
    int pad_;
} ffc_conv_seg;

typedef struct ffc_conv_phase {
    int py, px;          /* output offset of the phase */
    int PH, PW;          /* phase grid extent */
    int K;               /* valid k-table rows */
    int Kpad;            /* rows rounded up to the 16-deep k chunk */
    long long a_off;     /* float offset of this phase's packed weights [Mpad][Kpad] */
    int kt_off;          /* int4 offset of this phase's k-table */
    int pad_;
} ffc_conv_phase;

typedef struct ffc_conv_job {
    ffc_conv_seg seg[FFC_MAX_SEG];
    ffc_conv_phase ph[FFC_MAX_PHASE];
    const float* A;      /* packed weights */
    const int* ktab;     /* int4 per k: {seg | ch<<4, off_y, off_x, ky | kx<<16}; seg 15 = pad */
    float* out;          /* (B, M, OH, OW) */
    const float* bias;   /* (M) or NULL (already summed over segments) */
    const float* addend; /* (B, M, OH, OW) added before stats/activation, or NULL */
    float* stats;        /* BN partial slab [slots*WN][M] float4 {n, mean, M2, 0}, or NULL */
    int nseg, nphase;
    int B, M, Mpad, OH, OW, Sy, Sx;
    int act;             /* FFC_ACT_*, applied in the epilogue (use IDENTITY when a BN follows) */
    float act_param;
    int pad_;
} ffc_conv_job;

/* tiles: device int4 per workgroup {job | phase<<8, m0, n0, stats_slot}; tile_cfg selects
 * the (BM, BN) instantiation: 0 = 128x128, 1 = 64x128, 2 = 32x256. */
int ffc_conv_forward(const ffc_conv_job* jobs, int njobs, const int* tiles, int ntiles,
                     int tile_cfg, void* stream);
/* number of BN slab rows each tile writes (waves along N) for a tile_cfg */
int ffc_conv_stat_rows_per_tile(int tile_cfg);

/* 1x1-only job (every segment kind 'pw' at the output resolution, no pool / gate, one phase,
 * stats == NULL) as a plain tiled GEMM: SpectralTransform conv1 / conv2
 * (layers/ffc/spectral_transform.py:52-53,70-71), the FU spectral mix conv_layer
 * (layers/ffc/fourier_unity.py:25,45) and their data gradients on the training path.  A is the
 * job's ffc_conv_pack output ([Mpad][Kpad], k = segment-major channel).  cfg selects the tile:
 * 0 = 128 x 128, 1 = 64 x 128, 2 = 64 x 64 (output channels x pixels);  ffc_pw_tiles returns the
 * workgroup count of a cfg (or -1). */
int ffc_pw_forward(const ffc_conv_job* job, int cfg, void* stream);
int ffc_pw_tiles(int M, int B, int Q, int cfg);

/* ---- LDS-patch variant (the hot path for FFCTranspose k4 s2 and strided convs) ----
 * A workgroup owns one M-tile of 32 output channels x a pixel block (NS samples x TR x TC
 * phase-grid pixels) x all phases.  For each 16-channel chunk of each segment the input patch
 * the block needs (NS x 16 x PR x PC, zero outside the input) is staged once in LDS; every
 * (phase, tap) B fragment is then read from that patch, so an input element is fetched from
 * HBM/L2 once per block instead of once per (phase, tap).  Requires the taps per phase of each
 * segment to divide 4 (ConvT k4 s2: 4; 1x1: 1), or 16 in a one-phase job (Conv2d k4 s2: the
 * discriminator's convs, FFCDiscriminator ffc1-3 (models/ffc_discriminator.py:27-30), and the
 * data gradient of every ConvT k4 s2), whose chunks are then 4 channels x 16 taps.  A is packed
 * with every segment's channels padded to a multiple of its chunk (k = (seg, ch, tap)); the
 * packed buffer needs >= 64 floats of tail padding
 * (groups of taps a phase does not use are loaded, not multiplied).  Tap offsets travel in the
 * phase descriptor (kernel arguments, no table in memory).  Per-thread staging holds at most 2048
 * units (16-byte groups when vec4, else floats) of NS x 16 x PR x PC. */
#define FFC_PATCH_CC 16
typedef struct ffc_convp_seg {
    const float* x;      /* (B, C, IH, IW), or (B, C, 2IH, 2IW) when pool=1 */
    const float* gate;   /* optional (B, C) multiplier */
    int C, Cpad, IH, IW;
    int mult_y, mult_x;  /* input coord = m*mult + off */
    int org_y, org_x;    /* patch origin relative to r0*mult_y / c0*mult_x (the minimum tap offset) */
    int PR, PC;          /* patch rows / LDS row length in floats (vec4: whole 16-byte groups from the
                          * row start rounded down to a multiple of 4) */
    int pool;
    int vec4;            /* 1: stage the patch in 16-byte groups (IW % 4 == 0, x 16-byte aligned) */
    int cc;              /* channels per chunk: 16 (taps 1, 2, 4) or 4 (16 taps) */
    int direct;          /* ffc_convq_forward only: 1 = a 1x1 segment at the output resolution whose B
                          * fragments are read straight from x (no patch); 0 = staged through LDS */
    int qrow, qsample;   /* ffc_convq_forward only: LDS pixel strides of a patch row / sample (>= PC,
                          * >= PR * qrow), padded so that the 16 lanes of a ds_read_b128 group hit 16
                          * distinct bank slots */
} ffc_convp_seg;

typedef struct ffc_convp_phase {
    int py, px, PH, PW;
    int Kpad;            /* sum over segments of Cpad * T[s] */
    int T[FFC_MAX_SEG];  /* taps of each segment in this phase (1, 2, 4 or 16, or 0) */
    int kseg[FFC_MAX_SEG];   /* k offset of each segment inside the phase's packed rows */
    int tap[FFC_MAX_SEG][8];    /* each segment's taps: (dy << 16) | dx from the patch origin (first 8) */
    int tap_h[FFC_MAX_SEG];     /* 16 taps: tap j + 8 = tap j + tap_h for j < 8 (same encoding) */
    long long a_off;     /* float offset of the phase's packed weights [Mpad][Kpad] */
} ffc_convp_phase;

typedef struct ffc_convp_job {
    ffc_convp_seg seg[FFC_MAX_SEG];
    ffc_convp_phase ph[4];
    const float* A;
    float* out;
    const float* bias;
    const float* addend;
    float* stats;        /* [pixel blocks * 4][M] float4 {n, mean, M2, 0}, or NULL */
    int nseg, nphase;
    int B, M, Mpad, OH, OW, Sy, Sx;
    int NS, TR, TC, nrb, ncb;   /* pixel block: NS samples x TR rows x TC cols; row/col blocks per sample */
    int act;
    float act_param;
    /* optional: A pre-split into three exact bf16 planes (hi, mid, lo: ffc_split_bf16), plane p at
     * A3 + p * a3_stride elements; NULL = split A in registers per chunk */
    const uint16_t* A3;
    long long a3_stride;
} ffc_convp_job;

/* tiles: int4 {job, m0, pixel block, 0}; cfg: 0 = 4 phases x 4 N-tiles/wave, 1 = 4 x 2,
 * 2 = 1 phase x 2 N-tiles/wave, 3 = 1 x 1; | FFC_CONVP_EXACT_F32 selects the f32-input MFMA
 * (bitwise fp32 fma chains) instead of the default fp32-accurate split-bf16 MFMA products */
#define FFC_CONVP_EXACT_F32 8

/* fp32 -> three exact bf16 planes by truncation (hi = top 8 significand bits, mid = the next 8 of
 * x - hi, lo = the rest): planes[p * stride + i], p = 0, 1, 2; stride >= n, a multiple of 8.
 * The pre-split packed weights of the split-bf16 patch conv (ffc_convp_job.A3). */
int ffc_split_bf16(const float* x, long long n, uint16_t* planes, long long stride, void* stream);
int ffc_convp_forward(const ffc_convp_job* jobs, int njobs, const int* tiles, int ntiles, int cfg,
                      void* stream);

/* Stride-2 transposed convolution jobs (4 phases, FFCTranspose's ConvTranspose2d k4 s2 p1 + the folded
 * SpectralTransform.conv2, layers/ffc/ffc_transpose.py:79-106, spectral_transform.py:108) with the
 * operands pre-split for the fp32-accurate split-bf16 MFMA products: each input element is split
 * into three bf16 pieces ONCE per workgroup while it is staged into LDS (ffc_convp_forward splits
 * every B fragment at every use).  Same ffc_convp_job, with: K order per segment = (16-channel
 * chunk, tap, channel); A3 (pre-split packed weights) required; staged segments' PR x PC = the
 * patch in pixels (PC = row length), cc = 16; direct segments (1x1 at the output resolution, 1 tap)
 * read B from global memory.  tiles: int4 {job, m0, pixel block, 0}, m0 in steps of 32 * MT.
 * cfg 0..3 -> (MT M-tiles of 32 channels, NTW N-tiles of 32 pixels) per wave via ffc_convq_config. */
int ffc_convq_config(int cfg, int* mt, int* ntw);
/* The A3 operand of ffc_convq_forward: the packed weights A (ffc_conv_pack, phases at a_off, rows Mpad,
 * Kpad per phase) split into three bf16 pieces and laid out in MFMA fragment order, element
 * 3 * a_off + ((mtile * Kpad/16 + kstep) * 3 + piece) * 512 + lane * 8 + j for
 * A[32 * mtile + (lane & 31)][16 * kstep + 8 * (lane >> 5) + j] (one 1 KiB coalesced load per fragment
 * piece); A3 holds 3 * (total A floats) elements, 16-byte aligned. */
int ffc_convq_pack_a3(const ffc_convp_job* job, const float* A, uint16_t* A3, void* stream);
int ffc_convq_forward(const ffc_convp_job* jobs, int njobs, const int* tiles, int ntiles, int cfg,
                      void* stream);
/* K-split variant (small batches: too few output tiles to fill 256 CUs).  Each output tile (slot)
 * runs as ksplit workgroups over contiguous ranges of its 16-channel chunks (staged segments, then
 * direct ones) that store fp32 partial fragments to part (ffc_convq_split_floats(cfg, nslots,
 * ksplit) floats, 16-byte aligned); a second launch adds each slot's partials in split order
 * (deterministic) and runs the epilogue.  tiles: ntiles = nslots * ksplit int4 {job, m0, pixel
 * block, slot * 8 + split}; slot_tiles: nslots int4 {job, m0, pixel block, 0} in slot order.
 * ksplit = 1 is ffc_convq_forward (slot_tiles / part unused). */
long long ffc_convq_split_floats(int cfg, int nslots, int ksplit);
int ffc_convq_forward_split(const ffc_convp_job* jobs, int njobs, const int* tiles, int ntiles,
                            const int* slot_tiles, int nslots, int cfg, int ksplit, float* part,
                            void* stream);

/* Weight packing for one job: A[phase][Mpad][Kpad] (zero padded), bias_out[M] = sum of
 * segment biases.  w_layout[s]: 0 = Conv2d (O, I, kh, kw), 1 = ConvTranspose2d (I, O, kh, kw).
 * ktab/phase tables as in ffc_conv_job (host job struct is passed by pointer). */
int ffc_conv_pack(const ffc_conv_job* job, const float* const* seg_weight, const int* w_layout,
                  const int* kh, const int* kw, const float* const* seg_bias,
                  float* A_out, float* bias_out, void* stream);

/* Dense GEMM + bias + activation: out[b][n] = act(sum_k A[b][k] Wt[k][n] + bias[n]), A (B, K),
 * Wt (K, N) row-major, K <= 256.  Columns [0, N0) go to out0 (B, N0), [N0, N) to out1 (B, N - N0).
 * Replaces ConvTranspose2d(k, 1, 0) on a 1x1 input (ffc_transpose.py:79-86 in the generator's first
 * layer, models/ffc_generator.py:24: n = (m, ky, kx)) and nn.Linear (fgan128_complete.py:453-455). */
int ffc_dense_forward(const float* A, const float* Wt, const float* bias, int B, int K, int N, int N0,
                      float* out0, float* out1, int act, float act_param, void* stream);

/* ------------------------------------------------------------------ batch norm
 * nn.BatchNorm2d semantics (train: biased var normalises, unbiased var -> running_var,
 * num_batches_tracked += 1, momentum<0 means cumulative average; eval: running stats).
 * Used for SpectralTransform.bn1 (spectral_transform.py:57,89), FourierUnitSN.bn
 * (fourier_unity.py:28,49) and FFC_BN_ACT.bn_l/bn_g (ffc_bn_act.py:49-60,73-81). */
/* merge a partial slab [nrows][C] float4 {n, mean, M2} into moments[C][3] = {n, sum, sumsq} (fp64).
 * ffc_bn_reduce and ffc_bn_reduce_finalize need ffc_bn_reduce_ws_doubles(nrows, C) more doubles of
 * scratch right behind moments[C][3] (nonzero for large slabs, >= 1024 rows, which are merged in two
 * coalesced launches: 16-channel x row-range partials, then a fixed-order merge per channel). */
size_t ffc_bn_reduce_ws_doubles(int nrows, int C);
int ffc_bn_reduce(const float* slab, int nrows, int C, double* moments, void* stream);
/* moments (possibly all-reduced across ranks) -> scale/shift; updates running stats */
int ffc_bn_finalize(const double* moments, int C, const float* gamma, const float* beta,
                    float* running_mean, float* running_var, int64_t* num_batches_tracked,
                    int use_batch_stats, int update_running, float momentum, float eps,
                    float count_mult, float* scale, float* shift, void* stream);
/* single-rank fusion of ffc_bn_reduce + ffc_bn_finalize (use_batch_stats = 1) */
int ffc_bn_reduce_finalize(const float* slab, int nrows, int C, double* moments, const float* gamma,
                           const float* beta, float* running_mean, float* running_var,
                           int64_t* num_batches_tracked, int update_running, float momentum, float eps,
                           float count_mult, float* scale, float* shift, void* stream);
/* y = act(x*scale[c] + shift[c]) elementwise (in place allowed) */
int ffc_bn_act_apply(const float* x, float* y, int B, int C, int HW, const float* scale,
                     const float* shift, int act, float act_param, void* stream);
/* y = act(x*scale[c] + shift[c]) + noise_w[c] * noise[b] (FFC_BN_ACT followed by the fgan128
 * NoiseInjection, fgan128_complete.py:496-515 / layers/noise_injection.py:25-32); noise (B, 1, H, W),
 * HW % 4 == 0, 16-byte aligned tensors; in place allowed */
int ffc_bn_act_noise_apply(const float* x, float* y, int B, int C, int HW, const float* scale,
                           const float* shift, int act, float act_param, const float* noise_w,
                           const float* noise, void* stream);

/* Batched forms for the BNs of one FFC layer (bn_l and bn_g come out of the same conv launch,
 * ffc_bn_act.py:80-83): up to FFC_MAX_BN_BATCH items per call, one launch for all of them where the
 * single forms would launch once per item (launch latency dominates these small kernels).  Each item
 * has the meaning of the single call's arguments. */
#define FFC_MAX_BN_BATCH 4
typedef struct ffc_bn_rf_item {       /* ffc_bn_reduce_finalize arguments */
    const float* slab;
    int nrows, C;
    double* moments;                  /* [C][3] + ffc_bn_reduce_ws_doubles(nrows, C) */
    const float* gamma;
    const float* beta;
    float* running_mean;
    float* running_var;
    int64_t* num_batches_tracked;
    int update_running;
    float momentum, eps, count_mult;
    float* scale;
    float* shift;
} ffc_bn_rf_item;
int ffc_bn_reduce_finalize_batch(const ffc_bn_rf_item* items, int n, void* stream);
typedef struct ffc_bn_apply_item {    /* ffc_bn_act_noise_apply arguments (noise_w / noise may be NULL) */
    const float* x;
    float* y;
    int B, C, HW;
    const float* scale;
    const float* shift;
    int act;
    float act_param;
    const float* noise_w;
    const float* noise;
    float* plane_sum;   /* optional [B][C][ffc_plane_chunks(HW)]: the sums of y over each chunk of each
                           plane (the SE means of the next layer without a second read of y); needs
                           HW % 4 == 0, HW >= 256 and 16-byte aligned x / y / noise */
} ffc_bn_apply_item;
int ffc_bn_act_apply_batch(const ffc_bn_apply_item* items, int n, void* stream);
int ffc_plane_chunks(int HW);
/* SELayer gate from ffc_bn_act_apply_batch's plane sums (spectral_transform.py:12-28):
 * mean[b][c] = sum_k sums[b][c][k] / HW (k < chunks, fixed order), then the FCs as ffc_se_gate. */
int ffc_se_gate_sums(const float* sums, int chunks, int B, int C, int HW, const float* w1, const float* w2,
                     int hidden, float* gate, void* stream);

/* ------------------------------------------------------------------ spectral branch
 * SELayer gate (spectral_transform.py:12-28): gate[b][c] = sigmoid(W2 relu(W1 mean_hw x)),
 * hidden may be 0 (gate = 0.5).  pool=1: mean over the 2x2-avg-pooled input. */
int ffc_se_gate(const float* x, int B, int C, int H, int W, int pool, const float* w1,
                const float* w2, int hidden, float* gate, void* stream);

/* Fused SpectralTransform prologue, one workgroup per sample (spectral_transform.py:79-89):
 * [2x2 avg pool] -> SE gate -> conv1 (1x1) -> t (B, c, h, w) and per-sample BN1 partials
 * slab [B][c] float4 {n, mean, M2}.  wconv1T: conv1 weight transposed by ffc_pack_transpose
 * ((Cin, ceil32(c))).  gate_out (B, Cin) optional.  The sample must fit in LDS:
 * ffc_st_prologue_lds_bytes() == 0 means "use ffc_se_gate + conv". */
size_t ffc_st_prologue_lds_bytes(int Cin, int H, int W, int pool, int hidden, int c);
int ffc_st_prologue(const float* x, int B, int Cin, int H, int W, int pool, const float* w1,
                    const float* w2, int hidden, const float* wconv1T, int c, float* t, float* slab,
                    float* gate_out, void* stream);
/* The same over `split` workgroups per sample, each taking 1/split of conv1's output tiles
 * (ceil32(c)/32 x ceil32(h*w)/32; split must divide that count) after its own pool + SE gate:
 * small batches fill the CUs.  slab gets [B * split][c] rows (row b * split + s; channels a
 * workgroup does not cover are {0, 0, 0}).  ffc_st_prologue_split() is the split the library
 * picks for a batch (1 when B alone fills the GPU). */
int ffc_st_prologue_split(int B, int Cin, int H, int W, int pool, int c);
int ffc_st_prologue_ex(const float* x, int B, int Cin, int H, int W, int pool, const float* w1,
                       const float* w2, int hidden, const float* wconv1T, int c, int split, float* t,
                       float* slab, float* gate_out, void* stream);
/* ffc_st_prologue_ex with conv1 on fp32-accurate split-bf16 MFMA products (three exact bf16
 * pieces per operand, six products: as the local convolutions) instead of the f32-input MFMA:
 * wc3 = ffc_st_pack_a3(conv1.weight (c, Cin)), ffc_st_pack_a3_elems(c, Cin) uint16 elements,
 * 16-byte aligned; Cin % 16 == 0 (0 elements: unsupported).  wc3 = NULL is ffc_st_prologue_ex. */
size_t ffc_st_pack_a3_elems(int c, int cin);
int ffc_st_pack_a3(const float* w, int c, int cin, uint16_t* wc3, void* stream);
int ffc_st_prologue_ex3(const float* x, int B, int Cin, int H, int W, int pool, const float* w1,
                        const float* w2, int hidden, const float* wconv1T, const uint16_t* wc3, int c, int split,
                        float* t, float* slab, float* gate_out, void* stream);
/* SpectralTransform conv1 with the SE gate for planes the fused prologue cannot hold
 * (spectral_transform.py:87-89): t[b,o,p] = sum_c w[o,c] * gate[b,c] * x[b,c,p], p < HW, plus
 * bn1 partials slab [B * ffc_pw_gate_blocks(HW)][M] float4 {n, mean, M2} (slab may be NULL).
 * w: conv1 weight (M, Cin); gate (B, Cin) or NULL.  ffc_pw_gate_lds_bytes() == 0: unsupported. */
int ffc_pw_gate_blocks(int HW);
size_t ffc_pw_gate_lds_bytes(int Cin, int M);
int ffc_pw_gate_conv(const float* x, const float* gate, const float* w, int B, int Cin, int M, int HW,
                     float* t, float* slab, void* stream);
/* wT[k][o] = w[o][k] for a row-major (R, K) matrix, o zero-padded to ceil32(R) */
int ffc_pack_transpose(const float* w, int R, int K, float* wT, void* stream);

/* Direct ConvTranspose2d(k=4, s=2, p=1) for M <= 4 output channels (the generator's last
 * layer, models/ffc_generator.py:28; ffc_transpose.py:96-100):
 *   out = act(conv_t(x0; w0) [+ conv_t(x1; w1)] + bias).
 * The weights are first packed by ffc_convt_smallm_pack from the raw ConvTranspose2d weights
 * w0 (C0, M, 4, 4) and w1 (C1, M, 4, 4) (w1 NULL with C1 = 0) into wpack
 * [ffc_convt_smallm_pack_floats(C0, C1)] = [C0 + C1][16 taps][4], 16-byte aligned; x1 may be NULL. */
size_t ffc_convt_smallm_pack_floats(int C0, int C1);
int ffc_convt_smallm_pack(const float* w0, int C0, const float* w1, int C1, int M, float* wpack, void* stream);
int ffc_convt_k4s2_smallm(const float* x0, int C0, const float* x1, int C1, const float* wpack,
                          const float* bias, int B, int IH, int IW, int M, float* out, int act,
                          float act_param, void* stream);
/* Direct Conv2d(k=3, s=1, p=1) for M <= 4 output channels (the fgan128 generator's head conv7,
 * fgan128_complete.py:484): out = act(conv(x0; w0) [+ conv(x1; w1)] + bias), (B, M, H, W).
 * w*: raw Conv2d weights (M, C, 3, 3); x1/w1 may be NULL. */
int ffc_conv3x3_smallm(const float* x0, int C0, const float* w0, const float* x1, int C1,
                       const float* w1, const float* bias, int B, int H, int W, int M, float* out,
                       int act, float act_param, void* stream);

/* Deferred input transform of one conv input segment: the producing FFC_BN_ACT's BatchNorm2d +
 * activation and the NoiseInjection that follows it (ffc_bn_act.py:80-83 then
 * noise_injection.py:25-32; fgan128_complete.py:509-513), applied while the consumer stages its
 * operand instead of in a separate pass:
 *   x' = act(x*scale[c] + shift[c]) [+ noise_w[c] * noise[b, y, x]]   (zero padding stays zero)
 * noise: (B, 1, H, W) or NULL (then noise_w is ignored). */
typedef struct ffc_in_tf {
    const float* scale;
    const float* shift;
    int act;
    float act_param;
    const float* noise_w;
    const float* noise;
} ffc_in_tf;

/* ffc_conv3x3_smallm over deferred inputs: segment s is read through tf_s (NULL: as stored).
 * Replaces the producer's ffc_bn_act_noise_apply pass + ffc_conv3x3_smallm (the fgan128 conv6 ->
 * conv7 hand-off); results match that pair to within 2e-6 normwise (this kernel's GELU uses the
 * A&S 7.1.26 erf, |error| <= 1.5e-7; the apply pass uses erff). */
int ffc_conv3x3_smallm_tf(const float* x0, int C0, const float* w0, const float* x1, int C1,
                          const float* w1, const float* bias, int B, int H, int W, int M, float* out,
                          int act, float act_param, const ffc_in_tf* tf0, const ffc_in_tf* tf1,
                          void* stream);

/* Fourier unit (FourierUnitSN.forward, fourier_unity.py:32-56), fused per sample:
 *   s   = in_relu ? relu(t*in_scale + in_shift) : t, nearest-upsampled by `up` (1|2)
 *         (SpectralTransform's bn1/act1 + Upsample, spectral_transform.py:44-45,79,89)
 *   Z   = rfftn(s, ortho) as interleaved Re/Im channels;  Y = Wmix Z  (1x1 conv_layer)
 *   pass 0: write per-sample BN partials of Y to stats_slab [B][2C] float4
 *   pass 1: out = (residual ? s : 0) + irfftn(relu(Y*bn_scale + bn_shift), s=(H,W), ortho)
 * wmixT: (2C, Mpad) transposed, zero-padded copy of conv_layer.weight (Mpad = ceil32(2C)).
 * H, W: powers of two in [4, 32] (the sizes of the FFC-DCGAN generator/discriminator). */
int ffc_fu_forward(const float* t, int B, int C, int H, int W, int up, const float* in_scale,
                   const float* in_shift, int in_relu, const float* wmixT, int pass,
                   float* stats_slab, const float* bn_scale, const float* bn_shift,
                   int residual, float* out, void* stream);
/* transposed zero-padded mix weight: wmixT[i][o] = w[o][i] (w: (2C, 2C, 1, 1)) */
int ffc_fu_pack_mix(const float* w, int C2, float* wmixT, void* stream);
/* LDS bytes the fused FU kernel needs (0 if unsupported) */
size_t ffc_fu_lds_bytes(int C, int H, int W);

/* A train-mode BatchNorm finalized inside the kernel that applies it (single rank: no all-reduce
 * between the batch-statistics merge and the finalize).  Each workgroup of the consumer merges
 * the producer's partial rows slab[nrows][C] float4 {n, mean, M2, 0} in a fixed order (bit-identical
 * scale / shift everywhere); workgroup 0 updates running_mean / running_var (unbiased variance
 * over n * count_mult samples, momentum < 0 = cumulative average), bumps num_batches_tracked
 * (update_running) and writes scale_out / shift_out when given.  Replaces ffc_bn_reduce_finalize
 * + passing its scale / shift. */
typedef struct ffc_bn_fold {
    const float* slab;
    int nrows, C;
    const float* gamma;
    const float* beta;
    float* running_mean;
    float* running_var;
    int64_t* num_batches_tracked;
    int update_running;
    float momentum, eps, count_mult;
    float* scale_out;
    float* shift_out;
    /* SyncBN (round 6): when non-NULL, [C][3] fp64 raw moments {n, sum x, sum x^2} already merged
     * over the ranks (ffc_bn_reduce + an all-reduce); slab / nrows are then unused and every
     * consumer workgroup finalizes from these instead of merging partial rows */
    const double* moments;
} ffc_bn_fold;

/* ffc_fu_forward with the BNs folded in and pass 1 fed from pass 0 (no recompute):
 *   in_fold (optional, pass 0): bn1 of SpectralTransform finalized in-kernel from its slab, used as
 *           (in_scale, in_shift), and written to in_fold->scale_out / shift_out (required) for pass 1
 *           and later kernels (pass 1 then takes them as in_scale / in_shift);
 *   mix_fold (optional, pass 1): the FU's own BN from pass 0's slab instead of bn_scale / bn_shift;
 *   yspill (optional, both passes): (B, 2C, H, W/2+1) floats: pass 0 stores the mix output Y there,
 *           pass 1 applies BN + ReLU to it instead of recomputing row R2C + column FFT + mix. */
int ffc_fu_forward_ex(const float* t, int B, int C, int H, int W, int up, const float* in_scale,
                      const float* in_shift, int in_relu, const float* wmixT, int pass, float* stats_slab,
                      const float* bn_scale, const float* bn_shift, int residual, float* out,
                      const ffc_bn_fold* in_fold, const ffc_bn_fold* mix_fold, float* yspill, void* stream);
/* ffc_fu_forward_ex with the mix weight also given pre-split (wmix3 from ffc_fu_pack_mix3, C % 8 == 0):
 * the spectral mix then runs on split-bf16 MFMA products (six bf16 MFMAs per 16-deep k-block, each
 * product within 2^-21 of the fp32 product) and reads each weight piece as one 16-byte fragment
 * instead of splitting wmixT in every tile.  wmix3 = NULL (or FFC_FU_MFMA=f32) is ffc_fu_forward_ex. */
int ffc_fu_forward_ex3(const float* t, int B, int C, int H, int W, int up, const float* in_scale,
                       const float* in_shift, int in_relu, const float* wmixT, const uint16_t* wmix3, int pass,
                       float* stats_slab, const float* bn_scale, const float* bn_shift, int residual, float* out,
                       const ffc_bn_fold* in_fold, const ffc_bn_fold* mix_fold, float* yspill, void* stream);
/* ffc_fu_forward_ex3 with pass 0 over `kgroups` (1 or 2) workgroups per sample, each holding only a
 * range of the half-spectrum columns (round 6: the whole-spectrum LDS planes capped pass 0 at one
 * workgroup per CU).  Same FourierUnitSN.forward (fourier_unity.py:32-56); kgroups = 2 needs wmix3,
 * yspill and ffc_fu_kgroups(B, C, H, W) == 2, and changes two buffer contracts, so pass 0 and pass 1
 * must be given the same value:
 *   stats_slab has ffc_fu_slab_rows(B, C, H, W, kgroups) rows (row g B + b: sample b, group g; the
 *              mix BN's fold / reduce merge them all);
 *   yspill keeps B x 2C x H(W/2+1) floats, each channel's bins ordered [group][row][column in group]. */
int ffc_fu_forward_ex4(const float* t, int B, int C, int H, int W, int up, const float* in_scale,
                       const float* in_shift, int in_relu, const float* wmixT, const uint16_t* wmix3, int pass,
                       float* stats_slab, const float* bn_scale, const float* bn_shift, int residual, float* out,
                       const ffc_bn_fold* in_fold, const ffc_bn_fold* mix_fold, float* yspill, int kgroups,
                       void* stream);
/* the library's bin-group count for this fused FU (2 where the split layout fits two workgroups per
 * CU and the pre-split mix applies; FFC_FU_KGROUPS=1 forces 1) and the pass-0 slab rows it implies */
int ffc_fu_kgroups(int B, int C, int H, int W);
int ffc_fu_slab_rows(int B, int C, int H, int W, int kgroups);
/* wmixT (ffc_fu_pack_mix) -> its split bf16 pieces in MFMA fragment order: ffc_fu_mix3_elems(C) uint16
 * (16-byte aligned); 0 when C % 8 != 0 */
size_t ffc_fu_mix3_elems(int C);
int ffc_fu_pack_mix3(const float* wmixT, int C, uint16_t* wmix3, void* stream);

/* Large-plane Fourier unit (FourierUnitSN.forward, fourier_unity.py:32-56, for planes whose
 * per-sample spectrum does not fit one workgroup's LDS: the fgan128 generator's 64x64 and
 * 128x128 FUs, fgan128_complete.py:474-485).  Square H = W, a power of two in [16, 128],
 * 2C <= 128, up in {1, 2}; (h, w) = (H/up, W/up) is the grid of t.  Three stages over HBM:
 *   ffc_fu2d_r2c: T = rfft2(s0) unnormalised, s0 = in_relu ? relu(t*in_scale + in_shift) : t;
 *                 T (B, C, h, w/2+1) complex64 (interleaved float2)
 *   ffc_fu2d_mix: X = rfftn(s, ortho) of s = s0 nearest-upsampled by `up`, rebuilt from T;
 *                 Y = Wmix Z (Z: X's interleaved Re/Im channels, :40-45);
 *                 pass 0: BN partial slab [ffc_fu2d_slab_rows()][2C] float4 {n, mean, M2}
 *                 pass 1: Y = relu(Y*bn_scale + bn_shift) -> (B, C, H, W/2+1) complex64
 *                 pass 0 with Y != NULL also stores the raw Y (no BN) there, for ffc_fu2d_c2r_bn:
 *                 the statistics and the values they normalise are then the same numbers
 *   ffc_fu2d_c2r: out = irfftn(Y, s=(H, W), ortho) (+ s when residual) -> (B, C, H, W)
 * wmixT as for ffc_fu_forward. */
int ffc_fu2d_supported(int C, int H, int W, int up);
int ffc_fu2d_slab_rows(int B, int C, int H, int W);
int ffc_fu2d_r2c(const float* t, int B, int C, int h, int w, const float* in_scale,
                 const float* in_shift, int in_relu, float* T, void* stream);
int ffc_fu2d_mix(const float* T, int B, int C, int H, int W, int up, const float* wmixT, int pass,
                 float* stats_slab, const float* bn_scale, const float* bn_shift, float* Y, void* stream);
/* fp16-operand variant of ffc_fu2d_mix (BASELINE config 5 "fp16 MFMA channel-mix"): the spectrum and
 * the weights are rounded to fp16, products accumulate in fp32 (v_mfma_f32_32x32x16_f16); C in
 * {16, 32, 64}.  wmix16 from ffc_fu_pack_mix_f16: fp16 [ceil32(2C)][2C] = conv_layer.weight rows. */
int ffc_fu_pack_mix_f16(const float* w, int C2, void* wmix16, void* stream);
int ffc_fu2d_mix_f16(const float* T, int B, int C, int H, int W, int up, const void* wmix16, int pass,
                     float* stats_slab, const float* bn_scale, const float* bn_shift, float* Y, void* stream);
/* Column-fused variant of pass 1 + C2R for H = W in {32, 64, 128} (C in {16, 32}, or {16, 32, 64} with
 * f16): ffc_fu2d_mix_cols writes Yc (B, C, W/2+1, H) complex64 = the inverse column FFT (over H,
 * unnormalised) of relu(Y*bn_scale + bn_shift) -- the mix's workgroups own whole columns, so the
 * column FFT runs beside the MFMAs; ffc_fu2d_c2r_rows then finishes irfftn (rows, Im of bins 0 and
 * W/2 ignored, ortho scale) + residual.  wmix: fp32 wmixT (f16 = 0) or the fp16 weight (f16 = 1). */
int ffc_fu2d_cols_supported(int C, int H, int W, int up, int f16);
int ffc_fu2d_mix_cols(const float* T, int B, int C, int H, int W, int up, const void* wmix, int f16,
                      const float* bn_scale, const float* bn_shift, float* Yc, void* stream);
int ffc_fu2d_c2r_rows(const float* Yc, int B, int C, int H, int W, const float* t, int up,
                      const float* in_scale, const float* in_shift, int in_relu, int residual, float* out,
                      void* stream);
int ffc_fu2d_c2r(const float* Y, int B, int C, int H, int W, const float* t, int up,
                 const float* in_scale, const float* in_shift, int in_relu, int residual, float* out,
                 void* stream);
/* ffc_fu2d_c2r from pass 0's raw Y: relu(Y*bn_scale[2c|2c+1] + bn_shift[..]) (fourier_unity.py:46-49)
 * applied as each plane is loaded, so the two-pass mix becomes one mix + this C2R. */
int ffc_fu2d_c2r_bn(const float* Y, int B, int C, int H, int W, const float* t, int up,
                    const float* in_scale, const float* in_shift, int in_relu, int residual,
                    const float* bn_scale, const float* bn_shift, float* out, void* stream);
/* The same two stages with their BatchNorm finalized in-kernel, one channel per consumer (replaces
 * the ffc_bn_reduce_finalize launch before each; SpectralTransform.bn1, spectral_transform.py:57,89,
 * and FourierUnitSN.bn, fourier_unity.py:46): every (sample, channel) workgroup merges its channel's
 * slab rows itself (ffc_bn_fold over C = the r2c's C, or 2C for the c2r's two spectral channels;
 * momentum >= 0); the workgroups of sample 0 update the running statistics and write scale_out /
 * shift_out (required for in_fold: the C2R's residual takes them as in_scale / in_shift). */
int ffc_fu2d_r2c_ex(const float* t, int B, int C, int h, int w, const float* in_scale,
                    const float* in_shift, int in_relu, const ffc_bn_fold* in_fold, float* T, void* stream);
int ffc_fu2d_c2r_fold(const float* Y, int B, int C, int H, int W, const float* t, int up,
                      const float* in_scale, const float* in_shift, int in_relu, int residual,
                      const ffc_bn_fold* bn_fold, float* out, void* stream);
/* ffc_fu2d_r2c_ex + ffc_fu2d_mix pass 0 with the raw-Y spill, in one launch, for small t planes
 * (h = H/up in {8, 16}, C in {16, 32}; ffc_fu2d_r2c_mix_supported): every mix workgroup recomputes
 * its sample's T in LDS (bn1 + ReLU, row and column FFTs) instead of reading it from the R2C's
 * output; bn1 folded from its whole slab when in_fold is given (workgroup 0 leads: running statistics,
 * scale_out / shift_out).  stats_slab has ffc_fu2d_slab_rows() rows, as for ffc_fu2d_mix; T is not
 * materialized.  Same results as the two launches up to fp32 rounding of the FFT order. */
int ffc_fu2d_r2c_mix_supported(int C, int H, int W, int up);
int ffc_fu2d_r2c_mix(const float* t, int B, int C, int H, int W, int up, const float* in_scale,
                     const float* in_shift, int in_relu, const ffc_bn_fold* in_fold, const float* wmixT,
                     float* stats_slab, float* Y, void* stream);

/* ------------------------------------------------------------------ fgan128 caller ops
 * NoiseInjection.forward(x, noise) (layers/noise_injection.py:25-32): out = x + weight[c]*noise[b]
 * x, out (B, C, H, W); weight (C); noise (B, 1, H, W); HW % 4 == 0; in place allowed. */
int ffc_noise_inject(const float* x, const float* weight, const float* noise, float* out, int B, int C,
                     int HW, void* stream);
/* NoiseInjection backward (training path): dweight[c] = sum over b, hw of dout[b, c, hw] * noise[b, hw]
 * (dx = dout needs no kernel).  dout (B, C, H, W), noise (B, 1, H, W), HW % 4 == 0; deterministic. */
int ffc_noise_wgrad(const float* dout, const float* noise, int B, int C, int HW, float* dweight, void* stream);
/* eval-mode output of fgan128 FGenerator (fgan128_complete.py:516-521): out = uint8(255*(x*0.5+0.5))
 * (the reference's clamp to the tensor's own min/max is the identity); n % 4 == 0 */
int ffc_quantize_u8(const float* x, unsigned char* out, long long n, void* stream);


/* ------------------------------------------------------------------ training path (config 3)
 * Backward of the FFC operator surface for custom-op autograd (torch.autograd.Function per
 * reference op; the reference differentiates through ATen).  Data gradients of every conv /
 * convT / 1x1 run on ffc_conv_forward / ffc_convp_forward with the adjoint segment and the
 * same weight tensor under the other layout; the entry points below cover the rest.
 * Workspaces (ws) are caller-owned scratch; S = number of splits (see ffc_reduce_splits). */

/* dx = dy * act'(.) for FFC_BN_ACT's activation (ffc_bn_act.py:63-67, ST act1, FU relu).
 * t is the activation OUTPUT for ReLU/LeakyReLU/Tanh/Sigmoid and its INPUT for GELU. */
int ffc_act_bwd(const float* t, const float* dy, float* dx, long long n, int act, float act_param, void* stream);
/* splits per channel for the per-channel reductions below (grid C x S) */
int ffc_reduce_splits(int B, int C, int HW);
/* BatchNorm2d batch moments (nn.BatchNorm2d train forward): moments[C][3] = {n, sum x, sum x^2}
 * in fp64, the input of ffc_bn_finalize; ws: S*C*2 doubles */
int ffc_channel_moments(const float* x, int B, int C, int HW, double* ws, int S, double* moments, void* stream);
/* BatchNorm2d (+ following activation) backward: y = act(x*scale + shift) with scale/shift from
 * ffc_bn_finalize.  Train (moments != NULL): dx = gamma*inv*(g - mean(g) - xhat*mean(g*xhat));
 * eval (rmean, rvar: running stats the forward used): dx = gamma*inv*g.  dgamma = sum g*xhat,
 * dbeta = sum g (either may be NULL), dx may be NULL.  ws: S*C*2 doubles, coef: C*3 floats. */
int ffc_bn_bwd(const float* x, const float* dy, int B, int C, int HW, const float* scale, const float* shift,
               int act, float act_param, const double* moments, const float* rmean, const float* rvar, float eps,
               const float* gamma, double* ws, int S, float* coef, float* dgamma, float* dbeta, float* dx,
               void* stream);
/* The same backward split for SyncBN (sharded training, torch.nn.SyncBatchNorm semantics):
 * ffc_bn_bwd_sums -> sums[C][2] = {sum g, sum g*x} of this rank (fp64, fixed order); the caller
 * all-reduces a copy; ffc_bn_bwd_coeff(global sums, global moments) -> coef for dx, and
 * ffc_bn_bwd_coeff(local sums, ...) -> this rank's dgamma / dbeta (coef scratch); then
 * ffc_bn_bwd_apply -> dx. */
int ffc_bn_bwd_sums(const float* x, const float* dy, int B, int C, int HW, const float* scale, const float* shift,
                    int act, float act_param, double* ws, int S, double* sums, void* stream);
int ffc_bn_bwd_coeff(const double* sums, int C, const double* moments, float eps, const float* gamma, float* coef,
                     float* dgamma, float* dbeta, void* stream);
int ffc_bn_bwd_apply(const float* x, const float* dy, int B, int C, int HW, const float* scale, const float* shift,
                     int act, float act_param, const float* coef, float* dx, void* stream);
/* Weight gradient of nn.Conv2d / nn.ConvTranspose2d / 1x1 conv / nn.Linear (ffc.py:45-70,
 * ffc_transpose.py:48-86, spectral_transform.py:23-28,52-71, fourier_unity.py:20-23):
 *   dW[m][n][kh][kw] = sum_b sum_q U[b][m][q] * V[b][n][qy*stride - pad + kh*dil][qx*stride - pad + kw*dil]
 * U (B, Mu, PH, PW), V (B, Nv, VH, VW), zero outside V.  Conv2d: U = dy, V = x -> (Cout, Cin, k, k);
 * ConvTranspose2d: U = x, V = dy -> (Cin, Cout, k, k).  Split-K: S even shares of the flattened
 * (sample, pixel) K, 1 <= S <= B*PH*PW, partials in ws (S * Mu * Nv*k*k floats; unused when S == 1
 * and accumulate == 0) summed in a fixed order (deterministic); accumulate adds into dW. */
/* output tile edge ffc_conv_wgrad uses for (Mu, NT = Nv*k*k): grid = ceil(NT/t) x ceil(Mu/t) x S */
int ffc_conv_wgrad_tile(int Mu, int NT);
int ffc_conv_wgrad(const float* U, int Mu, int PH, int PW, const float* V, int Nv, int VH, int VW, int B, int k,
                   int stride, int pad, int dil, int S, float* ws, float* dW, int accumulate, void* stream);
/* rfftn(x, dim=(-2,-1), norm="ortho") of P planes (P, H, W) into the interleaved Re/Im planes of
 * fourier_unity.py:38-42: Re of plane p at Z[2p], Im at Z[2p+1], each H x (W/2+1).  Bins with a
 * Hermitian mirror (0 < kw, 2kw != W) are multiplied by interior_scale (2: the adjoint of irfftn).
 * Square power-of-two planes 8..128 run on the line FFTs of the staged Fourier unit; other planes
 * (H, W <= 64) on direct DFTs. */
int ffc_rfft2_planes(const float* x, int P, int H, int W, float interior_scale, float* Z, void* stream);
/* irfftn(X, s=(H,W), dim=(-2,-1), norm="ortho") (fourier_unity.py:51-56) from interleaved planes,
 * Im of the kw = 0 and kw = W/2 bins ignored, mirrored bins x interior_scale (0.5: the adjoint of
 * rfftn), + addend (P, H, W) when not NULL (SpectralTransform's x + fu(x), :108).  Square
 * power-of-two planes 16..128 on line FFTs, other planes (H, W <= 64) on direct DFTs. */
int ffc_irfft2_planes(const float* Z, int P, int H, int W, float interior_scale, const float* addend, float* y,
                      void* stream);
/* SELayer backward (spectral_transform.py:23-28): dx, plus the per-sample vectors of the two
 * Linear weight gradients: dpre2 (B, C), hact (B, hidden), dpre1 (B, hidden), mean (B, C).
 * hidden = C // 16 may be 0 (gate 0.5).  ws: 4 * B * C floats of scratch (per-plane sums, gate,
 * mean gradient); three launches (plane sums over the whole chip, per-sample gate, dx). */
int ffc_se_bwd(const float* x, const float* dout, int B, int C, int H, int W, const float* w1, const float* w2,
               int hidden, float* dx, float* dpre2, float* hact, float* dpre1, float* mean, float* ws, void* stream);
/* Conv2d whose kernel covers the whole input plane (k == H == W, padding 0 -> 1x1 output) with
 * M <= 4 outputs, up to two summed segments (FFCDiscriminator's last FFC_BN_ACT, 4x4 -> 1x1 + Sigmoid,
 * models/ffc_discriminator.py:31; ffc.py:89-97): out[b][m] = act(sum x_s[b][k] w_s[m][k] + bias[m]),
 * K_s = C_s*k*k, weights in nn.Conv2d layout; 16-byte aligned operands */
int ffc_conv_full_smallm(const float* x0, int K0, const float* w0, const float* x1, int K1, const float* w1,
                         const float* bias, int B, int M, float* out, int act, float act_param, void* stream);
/* y = scale * (2x2 window sum) of P planes (H, W even): AvgPool2d(2,2) with scale 0.25
 * (spectral_transform.py:46-47), the adjoint of nearest Upsample(x2) with scale 1 */
int ffc_pool2(const float* x, long long P, int H, int W, float scale, float* y, void* stream);
/* y = scale * nearest x2 upsample of P planes (h, w): Upsample(scale_factor=2) with scale 1
 * (spectral_transform.py:44-45), the adjoint of AvgPool2d(2,2) with scale 0.25 */
int ffc_up2(const float* x, long long P, int h, int w, float scale, float* y, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* FFC_AMD_H */
