// Caller-level elementwise ops of the fgan128 generator (gfx950):
//   NoiseInjection.forward (layers/noise_injection.py:25-32): out = x + weight[c] * noise[b, hw]
//   eval-mode output quantization (fgan128_complete.py:516-521): u8 = uint8(255 * (x * 0.5 + 0.5))
// Both are HBM-bound streams: float4 per lane, grid-stride.
#include "ffc_internal.h"

namespace {

__global__ void noise_inject_kernel(const float4* __restrict__ x, const float* __restrict__ w,
                                    const float4* __restrict__ noise, float4* __restrict__ out, int C, int HW4,
                                    long long n4) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
        const long long bc = i / HW4;
        const int p = (int)(i - bc * HW4);
        const int b = (int)(bc / C), c = (int)(bc - (long long)b * C);
        const float wc = w[c];
        const float4 v = x[i];
        const float4 n = noise[(long long)b * HW4 + p];
        out[i] = make_float4(fmaf(wc, n.x, v.x), fmaf(wc, n.y, v.y), fmaf(wc, n.z, v.z), fmaf(wc, n.w, v.w));
    }
}

__device__ __forceinline__ unsigned int q8(float x) {
    // torch: 255 * (x * 0.5 + 0.5) in fp32 (x * 0.5 is exact, so the fused form rounds identically),
    // then a truncating float -> uint8 conversion
    const float v = 255.0f * fmaf(x, 0.5f, 0.5f);
    return (unsigned int)(int)v & 0xFFu;
}

__global__ void quantize_u8_kernel(const float4* __restrict__ x, unsigned int* __restrict__ out, long long n4) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
        const float4 v = x[i];
        out[i] = q8(v.x) | (q8(v.y) << 8) | (q8(v.z) << 16) | (q8(v.w) << 24);
    }
}

// NoiseInjection backward, weight: dw[c] = sum_{b, hw} g[b, c, hw] * noise[b, hw].  One block per
// channel, fp64 per-thread sums over (b, hw) in a fixed stride, a fixed shuffle tree, the waves in
// order: deterministic.
__global__ __launch_bounds__(256) void noise_wgrad_kernel(const float4* __restrict__ g, const float4* __restrict__ noise,
                                                          int B, int C, int HW4, float* __restrict__ dw) {
    const int c = blockIdx.x;
    double acc = 0.0;
    for (int b = 0; b < B; ++b) {
        const float4* gp = g + ((size_t)b * C + c) * HW4;
        const float4* np = noise + (size_t)b * HW4;
        for (int i = threadIdx.x; i < HW4; i += 256) {
            const float4 u = gp[i], n = np[i];
            acc += (double)u.x * n.x + (double)u.y * n.y + (double)u.z * n.z + (double)u.w * n.w;
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
    __shared__ double part[4];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) dw[c] = (float)(((part[0] + part[1]) + part[2]) + part[3]);
}

int grid_for(long long n4) {
    const long long g = (n4 + 255) / 256;
    return (int)(g < 8192 ? (g > 0 ? g : 1) : 8192);
}

}  // namespace

extern "C" int ffc_noise_inject(const float* x, const float* weight, const float* noise, float* out, int B, int C,
                                int HW, void* stream) {
    FFC_CHECK_ARG(x && weight && noise && out, "ffc_noise_inject: null pointer");
    FFC_CHECK_ARG(B > 0 && C > 0 && HW > 0 && HW % 4 == 0, "ffc_noise_inject: HW must be a positive multiple of 4");
    const long long n4 = (long long)B * C * (HW / 4);
    hipLaunchKernelGGL(noise_inject_kernel, dim3(grid_for(n4)), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const float4*>(x), weight, reinterpret_cast<const float4*>(noise),
                       reinterpret_cast<float4*>(out), C, HW / 4, n4);
    return ffc::launch_status("ffc_noise_inject");
}

extern "C" int ffc_quantize_u8(const float* x, unsigned char* out, long long n, void* stream) {
    FFC_CHECK_ARG(x && out && n > 0 && n % 4 == 0, "ffc_quantize_u8: n must be a positive multiple of 4");
    const long long n4 = n / 4;
    hipLaunchKernelGGL(quantize_u8_kernel, dim3(grid_for(n4)), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const float4*>(x), reinterpret_cast<unsigned int*>(out), n4);
    return ffc::launch_status("ffc_quantize_u8");
}

extern "C" int ffc_noise_wgrad(const float* g, const float* noise, int B, int C, int HW, float* dw, void* stream) {
    FFC_CHECK_ARG(g && noise && dw, "ffc_noise_wgrad: null pointer");
    FFC_CHECK_ARG(B > 0 && C > 0 && HW > 0 && HW % 4 == 0, "ffc_noise_wgrad: HW must be a positive multiple of 4");
    hipLaunchKernelGGL(noise_wgrad_kernel, dim3(C), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const float4*>(g), reinterpret_cast<const float4*>(noise), B, C, HW / 4, dw);
    return ffc::launch_status("ffc_noise_wgrad");
}
