// EXPERIMENT, not built into libffc_amd.so: the parity-split C2R of round 3, measured
// slower than fu2d_c2r_kernel on MI355X (fgan128 B = 512: 128^2 C2R 570 -> 682 us, 64^2 114 -> 169 us,
// profiles/r03/s2a).  Kept as an excerpt of csrc/fu2d_kernels.hip at round 3 (it needs that file's
// helpers: Split, LaneTw, stage_a / stage_b, zstride, in_tf, C2rArgs); the dispatch that selected it
// under FFC_C2R_FOLD=64|128 is at the end of this file.

// ---------------------------------------------------------------- stage 3 split over output-row parity
#ifndef FFC_C2R_FOLD_RPRE
#define FFC_C2R_FOLD_RPRE 0
#endif
// fu2d_c2r_kernel keeps a whole H x (W/2+1) complex plane in LDS (66.5 KB at 128^2: two workgroups per
// CU, whose load / FFT / store phases overlap only with each other).  Here each plane runs as two
// workgroups with half the LDS (four per CU): part p computes the output rows y = 2r + p.  With
// w = e^{+2 pi i / H} the inverse DFT over the rows splits as
//     x[2r]     = sum_{k < H/2} (Y[k] + Y[k + H/2])       w^{2rk}    (E: a length-H/2 IDFT)
//     x[2r + 1] = sum_{k < H/2} (Y[k] - Y[k + H/2]) w^k  w^{2rk}    (O: a length-H/2 IDFT)
// so each part loads the whole Y plane, folds it into H/2 rows while it goes to LDS (after the BN +
// ReLU of a spilled Y), runs length-H/2 column IFFTs (the packed DC / Nyquist column as in
// fu2d_c2r_kernel: Re(IDFT(a)) = IDFT of a's Hermitian part for any sequence) and the row C2R of its
// H/2 rows.  Blocks b and b + 8 are the two parts of one plane: the dispatcher deals blocks to the 8
// XCDs round robin, so both run on one XCD and the second read of Y and t is an L2 hit.
template <int H, int W, int UP>
__global__ __launch_bounds__(FU2_THREADS, 4) void fu2d_c2r_fold_kernel(C2rArgs a) {
    constexpr int HH = H / 2;
    constexpr int WP = W / 2 + 1;
    constexpr int ZS = zstride(WP);
    constexpr int N1 = Split<W>::N1, N2 = Split<W>::N2, Q = Split<W>::Q;
    static_assert(H <= 128 && HH % 2 == 0 && (HH * WP) % 2 == 0, "fold split");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float2* Z = reinterpret_cast<float2*>(smem);
    const int bid = blockIdx.x;
    const int part = (bid >> 3) & 1;
    const int plane = ((bid >> 4) << 3) | (bid & 7);
    const int ch = plane % a.C;
    const int tid = threadIdx.x;

    const float sc = a.in_scale ? a.in_scale[ch] : 1.0f;
    const float sh = a.in_scale ? a.in_shift[ch] : 0.0f;
    constexpr int tW = W / UP;
    const float* tpl = a.t + (size_t)plane * (H / UP) * tW;
    float* opl = a.out + (size_t)plane * H * W;
    constexpr int RLPR = FU2_THREADS / N1;                      // row pairs per round
    constexpr int RROUNDS = (HH / 2 + RLPR - 1) / RLPR;
    constexpr int RITER = (2 * W / 4 + N1 - 1) / N1;            // float4 outputs per thread per row pair
    constexpr bool RPRE = FFC_C2R_FOLD_RPRE && UP == 2;   // residual t prefetched with Y (16 VGPRs live throughout)
    float2 res[RPRE ? RROUNDS : 1][RPRE ? RITER : 1];
    {
        const bool bn = a.bn_scale != nullptr;
        const float bsr = bn ? a.bn_scale[2 * ch] : 1.0f, bhr = bn ? a.bn_shift[2 * ch] : 0.0f;
        const float bsi = bn ? a.bn_scale[2 * ch + 1] : 1.0f, bhi = bn ? a.bn_shift[2 * ch + 1] : 0.0f;
        constexpr int N4h = HH * WP / 2;                          // float4 (two bins) per half plane
        constexpr int NL = (N4h + FU2_THREADS - 1) / FU2_THREADS;
        const float4* src4 = reinterpret_cast<const float4*>(a.Y) + (size_t)plane * (2 * N4h);
        float4 v0[NL], v1[NL];
#pragma unroll
        for (int u = 0; u < NL; ++u) {
            const int i = u * FU2_THREADS + tid;
            const int ii = i < N4h ? i : 0;
            v0[u] = src4[ii];
            v1[u] = src4[ii + N4h];
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
                        const bool ok = g < HH / 2 && q4 < 2 * W / 4;
                        // output row 4g + 2rr + part reads t row 2g + rr
                        res[rd][i] = *reinterpret_cast<const float2*>(tpl + (ok ? (2 * g + rr) * tW + x / 2 : 0));
                    }
                }
            }
        }
        auto bnf = [&](float2 z) {
            return bn ? make_float2(fmaxf(fmaf(z.x, bsr, bhr), 0.0f), fmaxf(fmaf(z.y, bsi, bhi), 0.0f)) : z;
        };
#pragma unroll
        for (int u = 0; u < NL; ++u) {
            const int i = u * FU2_THREADS + tid;
            if (i < N4h) {
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const float2 z0 = bnf(e ? make_float2(v0[u].z, v0[u].w) : make_float2(v0[u].x, v0[u].y));
                    const float2 z1 = bnf(e ? make_float2(v1[u].z, v1[u].w) : make_float2(v1[u].x, v1[u].y));
                    const int f = 2 * i + e, r = f / WP, k = f - r * WP;
                    float2 z;
                    if (part == 0) {
                        z = make_float2(z0.x + z1.x, z0.y + z1.y);
                    } else {   // (Y[r] - Y[r + H/2]) e^{+2 pi i r / H}
                        const float dx = z0.x - z1.x, dy = z0.y - z1.y;
                        const float c = c_twc[r * (128 / H)], s = c_tws[r * (128 / H)];
                        z = make_float2(dx * c - dy * s, dx * s + dy * c);
                    }
                    Z[r * ZS + k] = z;
                }
            }
        }
    }
    __syncthreads();

    // packed DC / Nyquist column (pad column WP) over the folded length-H/2 columns, then the IFFTs
    static_assert(ZS > WP, "pad column for the packed DC / Nyquist column");
    for (int r = tid; r < HH; r += FU2_THREADS) {
        const int rm = (HH - r) & (HH - 1);
        const float2 a0 = Z[r * ZS], a1 = Z[rm * ZS], b0 = Z[r * ZS + W / 2], b1 = Z[rm * ZS + W / 2];
        const float ahx = 0.5f * (a0.x + a1.x), ahy = 0.5f * (a0.y - a1.y);
        const float bhx = 0.5f * (b0.x + b1.x), bhy = 0.5f * (b0.y - b1.y);
        Z[r * ZS + WP] = make_float2(ahx - bhy, ahy + bhx);
    }
    __syncthreads();
    {
        constexpr int N1c = Split<HH>::N1, LPR = FU2_THREADS / N1c;
        const int jj = tid % N1c;
        const LaneTw<HH> twc(jj);   // twiddles loaded per pass: not live across the Y loads
        for (int l0 = 0; l0 < W / 2; l0 += LPR) {
            const int l = l0 + tid / N1c;
            if (l < W / 2) line_fft<HH, true>(Z + (l == 0 ? WP : l), ZS, jj, twc);
        }
    }
    __syncthreads();

    // rows two at a time (local rows 2g, 2g+1 = output rows 4g + part, 4g + 2 + part), as in fu2d_c2r_kernel
    {
        const int jj = tid % N1;
        const LaneTw<W> twr(jj);
#pragma unroll
        for (int rd = 0; rd < RROUNDS; ++rd) {
            const int g = rd * RLPR + tid / N1;
            if (g < HH / 2) {
                float2* ra = Z + 2 * g * ZS;
                float2* rb = ra + ZS;
                float re[N2], im[N2];
#pragma unroll
                for (int m = 0; m < N2; ++m) {
                    const int k = jj + N1 * m;
                    float2 A, B;
                    if (k == 0 || k == W / 2) {
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
                stage_a<W, true>(re, im, twr);
                float ore[Q][N1], oim[Q][N1];
                stage_b<W, true>(ra, 1, re, im, jj, ore, oim);
                float* fa = reinterpret_cast<float*>(ra);
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
                for (int i = 0; i < RITER; ++i) {
                    const int q4 = jj + N1 * i;
                    if (q4 < 2 * W / 4) {
                        const int rr = q4 / (W / 4);
                        const int x = 4 * (q4 % (W / 4));
                        const int y = 4 * g + 2 * rr + part;
                        float4 v = *reinterpret_cast<const float4*>(fa + rr * W + x);
                        v.x *= a.norm;
                        v.y *= a.norm;
                        v.z *= a.norm;
                        v.w *= a.norm;
                        if (a.residual) {
                            if constexpr (UP == 1) {
                                const float4 s = *reinterpret_cast<const float4*>(tpl + (size_t)y * tW + x);
                                v.x += in_tf(s.x, sc, sh, a.in_relu);
                                v.y += in_tf(s.y, sc, sh, a.in_relu);
                                v.z += in_tf(s.z, sc, sh, a.in_relu);
                                v.w += in_tf(s.w, sc, sh, a.in_relu);
                            } else {
                                float2 s;
                                if constexpr (RPRE) s = res[rd][i];
                                else s = *reinterpret_cast<const float2*>(tpl + (size_t)(2 * g + rr) * tW + x / 2);
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


// ---- host-side selection (was in fu2d_kernels.hip; fu2d_c2r_launch took it for H >= c2r_fold_min()
// with B * C a multiple of 8, launching 2 * B * C workgroups with (H / 2) * zstride(W / 2 + 1) * 8 bytes
// of LDS)
C2rKernel pick_c2r_fold(int H, int W, int up) {
    if (H != W) return nullptr;
    switch (H) {
        case 64: return up == 1 ? fu2d_c2r_fold_kernel<64, 64, 1> : fu2d_c2r_fold_kernel<64, 64, 2>;
        case 128: return up == 1 ? fu2d_c2r_fold_kernel<128, 128, 1> : fu2d_c2r_fold_kernel<128, 128, 2>;
    }
    return nullptr;
}
// smallest plane that takes the parity-split C2R (FFC_C2R_FOLD=64 / =128); off by default: measured
// slower on fgan128 B = 512 (gpurun_out s2a, profiles/r03/s2a): 128^2 C2R 570 -> 682 us, 64^2 114 -> 169 us
// -- the second part's read of Y does not come from L2 often enough to pay for the doubled loads
int c2r_fold_min() {
    static const int v = [] {
        const char* e = std::getenv("FFC_C2R_FOLD");
        const int n = e ? std::atoi(e) : 0;
        return n <= 0 ? 1 << 30 : n;
    }();
    return v;
}


// ---- numpy emulation of the kernel's fold arithmetic (was tests/test_fu2d_cpu.py::test_c2r_parity_fold):
// @pytest.mark.parametrize("H", [64, 128])
// def test_c2r_parity_fold(H):
//     """fu2d_c2r_fold_kernel: part p of a plane computes output rows 2r + p from the folded half plane
//     E[k] = Y[k] + Y[k + H/2] (p = 0) or O[k] = (Y[k] - Y[k + H/2]) e^{+2 pi i k/H} (p = 1), each with
//     length-H/2 column IFFTs, the packed DC / Nyquist column on the folded columns and the row C2R --
//     numpy emulation of the kernel's index and twiddle arithmetic against irfftn(Y, s=(H, W))"""
//     W = H
//     HH = H // 2
//     rng = np.random.default_rng(7 * H)
//     Y = rng.standard_normal((H, W // 2 + 1)) + 1j * rng.standard_normal((H, W // 2 + 1))
//     # the kernel's twiddle: c_twc / c_tws[r * (128 / H)] = cos / sin(2 pi r / H)
//     tw = np.cos(2 * np.pi * np.arange(HH) / H) + 1j * np.sin(2 * np.pi * np.arange(HH) / H)
//     out = np.empty((H, W))
//     for part in (0, 1):
//         F = Y[:HH] + Y[HH:] if part == 0 else (Y[:HH] - Y[HH:]) * tw[:, None]
//         cols = np.fft.ifft(F, axis=0) * HH
//         a, b = F[:, 0], F[:, W // 2]
//         neg = (-np.arange(HH)) % HH
//         zc = np.fft.ifft(0.5 * (a + np.conj(a[neg])) + 1j * 0.5 * (b + np.conj(b[neg]))) * HH
//         cols[:, 0] = zc.real
//         cols[:, W // 2] = zc.imag
//         edge = np.arange(W // 2 + 1) % (W // 2) == 0
//         rows = np.fft.irfft(np.where(edge, cols.real, cols), n=W, axis=1) * W
//         out[part::2] = rows
//     ref = np.fft.irfftn(Y, s=(H, W)) * H * W
//     np.testing.assert_allclose(out, ref, rtol=0, atol=1e-9 * np.abs(ref).max())
