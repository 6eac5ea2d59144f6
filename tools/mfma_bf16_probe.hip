// Microbenchmark: achieved v_mfma_f32_32x32x16_bf16 rate on the whole chip (MI355X), MFMA only and
// with the convq inner loop's operand traffic (3 ds_read_b128 per 6 MFMAs).  Diagnostic only.
// hipcc -O3 --offload-arch=gfx950 tools/mfma_bf16_probe.hip -o /tmp/mfma_bf16_probe && /tmp/mfma_bf16_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int MODE, int NT, int ITERS>
__global__ __launch_bounds__(256, 2) void probe(float* out, int salt) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    for (int i = threadIdx.x; i < 4096; i += 256) reinterpret_cast<unsigned*>(lds)[i] = (unsigned)(i * 2654435761u + salt) & 0x3f803f80u;
    __syncthreads();
    floatx16 acc[NT];
    for (int n = 0; n < NT; ++n)
        for (int r = 0; r < 16; ++r) acc[n][r] = 0.0f;
    const int lane = threadIdx.x & 63;
    u32x4 av = {0x3f803f80u + lane, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u};
    u32x4 bv[NT];
    for (int n = 0; n < NT; ++n) bv[n] = av + (unsigned)n;
    int off = lane * 48;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int q = 0; q < 6; ++q) {
#pragma unroll
            for (int n = 0; n < NT; ++n) {
                if (MODE == 1 && q < 3) bv[n] = *reinterpret_cast<const u32x4*>(lds + ((off + n * 1536 + q * 16) & 16383));
                acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, av),
                                                                 __builtin_bit_cast(bf16x8, bv[n]), acc[n], 0, 0, 0);
            }
        }
        off += 48 * 64;
    }
    float s = 0.0f;
    for (int n = 0; n < NT; ++n)
        for (int r = 0; r < 16; ++r) s += acc[n][r];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE, int NT>
void run(int blocks) {
    constexpr int ITERS = 2000;
    float* out;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    probe<MODE, NT, ITERS><<<blocks, 256, 16384>>>(out, 1);
    hipEventRecord(e0);
    probe<MODE, NT, ITERS><<<blocks, 256, 16384>>>(out, 2);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = (double)blocks * 4 * ITERS * 6 * NT * 32768.0;
    printf("mode %d NT %d blocks %d: %.3f ms, %.1f TF/s (bf16 dense peak 2500)\n", MODE, NT, blocks, ms, flops / ms / 1e9);
    hipFree(out);
}

int main() {
    run<0, 4>(256);
    run<0, 4>(512);
    run<0, 4>(1024);
    run<1, 4>(512);
    run<0, 2>(512);
    run<1, 2>(512);
    return 0;
}
