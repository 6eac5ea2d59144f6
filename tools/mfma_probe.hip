// Microbenchmark: f32 MFMA issue rate with B operands fed from LDS, as in convp's inner loop.
// hipcc -O3 --offload-arch=gfx950 tools/mfma_probe.hip -o /tmp/mfma_probe && /tmp/mfma_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

// MODE 0: MFMA only (B from registers); MODE 1: one ds_read_b32 per MFMA (NT reads per step)
template <int MODE, int NT, int ITERS>
__global__ __launch_bounds__(256) void probe32(float* out, int salt) {
    __shared__ float lds[8192];
    for (int i = threadIdx.x; i < 8192; i += 256) lds[i] = (float)((i * 7 + salt) & 15) * 0.01f;
    __syncthreads();
    floatx16 acc[NT];
    for (int n = 0; n < NT; ++n)
        for (int r = 0; r < 16; ++r) acc[n][r] = 0.0f;
    const int lane = threadIdx.x & 63;
    float a = 0.001f * lane;
    float b[NT];
    for (int n = 0; n < NT; ++n) b[n] = 0.002f * (lane + n);
    int off = lane;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
#pragma unroll
            for (int n = 0; n < NT; ++n) {
                float bv = b[n];
                if (MODE == 1) bv = lds[(off + n * 32 + s * 129) & 8191];
                acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv, acc[n], 0, 0, 0);
            }
        }
        off += 7;
    }
    float s = 0.0f;
    for (int n = 0; n < NT; ++n)
        for (int r = 0; r < 16; ++r) s += acc[n][r];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

// 16x16x4 f32: B fragment lane l: B[k = l>>4][j = l&15]
template <int MODE, int NT, int ITERS>
__global__ __launch_bounds__(256) void probe16(float* out, int salt) {
    __shared__ float lds[8192];
    for (int i = threadIdx.x; i < 8192; i += 256) lds[i] = (float)((i * 7 + salt) & 15) * 0.01f;
    __syncthreads();
    floatx4 acc[NT];
    for (int n = 0; n < NT; ++n)
        for (int r = 0; r < 4; ++r) acc[n][r] = 0.0f;
    const int lane = threadIdx.x & 63;
    float a = 0.001f * lane;
    float b[NT];
    for (int n = 0; n < NT; ++n) b[n] = 0.002f * (lane + n);
    int off = lane;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
#pragma unroll
            for (int n = 0; n < NT; ++n) {
                float bv = b[n];
                if (MODE == 1) bv = lds[(off + n * 16 + s * 129) & 8191];
                acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv, acc[n], 0, 0, 0);
            }
        }
        off += 7;
    }
    float s = 0.0f;
    for (int n = 0; n < NT; ++n)
        for (int r = 0; r < 4; ++r) s += acc[n][r];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <typename K>
void run(const char* name, K k, int blocks, double flop_per_block) {
    float* out;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 1);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, i);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-40s blocks=%5d  %8.1f TF/s\n", name, blocks, flop_per_block * blocks * 10 / (ms * 1e-3) / 1e12);
    hipFree(out);
}

int main() {
    constexpr int IT = 256;
    const double f32 = 4.0 * 8 * IT * 2.0 * 32 * 32 * 2;   // per wave: NT*8*IT MFMAs x 4096 flop; x4 waves
    for (int blocks : {256, 512, 1024, 2048}) {
        run("32x32x2 regs NT=1", probe32<0, 1, IT>, blocks, 4 * 8.0 * IT * 1 * 4096);
        run("32x32x2 regs NT=2", probe32<0, 2, IT>, blocks, 4 * 8.0 * IT * 2 * 4096);
        run("32x32x2 regs NT=4", probe32<0, 4, IT>, blocks, 4 * 8.0 * IT * 4 * 4096);
        run("32x32x2 lds  NT=4", probe32<1, 4, IT>, blocks, 4 * 8.0 * IT * 4 * 4096);
        run("32x32x2 lds  NT=2", probe32<1, 2, IT>, blocks, 4 * 8.0 * IT * 2 * 4096);
        run("16x16x4 regs NT=8", probe16<0, 8, IT>, blocks, 4 * 8.0 * IT * 8 * 2048);
        run("16x16x4 lds  NT=8", probe16<1, 8, IT>, blocks, 4 * 8.0 * IT * 8 * 2048);
    }
    (void)f32;
    return 0;
}
