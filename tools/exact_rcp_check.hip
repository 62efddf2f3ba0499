// Exhaustive check of short correctly-rounded reciprocal sequences against the IEEE divide
// (DIAGNOSTIC for DESIGN.md §Numerics).  For every one of the 2^32 float bit patterns x:
//   f32: rcp_f32(x) = fma(fma(-x, r, 1), r, r), r = v_rcp_f32(x)        vs  1.0f / x
//   f64: rcp_f64(x) = two Newton steps from v_rcp_f64((double)x)        vs  1.0 / (double)x
//        (the product's rcp_d, cpt_device.hpp)
// Prints the mismatch counts and a few mismatching inputs per exponent range.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-gpu-flush-denormals-to-zero \
//         -fhip-fp32-correctly-rounded-divide-sqrt tools/exact_rcp_check.hip -o build/exact_rcp_check
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ float rcp_f32(float x) {
    const float r = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}

// the product's rcp_d (cpt_device.hpp): two Newton steps, v_rcp_f64's value where they make NaN
__device__ __forceinline__ double rcp_f64(float xf) {
    const double x = (double)xf;
    const double r0 = __builtin_amdgcn_rcp(x);
    double e = __builtin_fma(-x, r0, 1.0);
    double r = __builtin_fma(r0, e, r0);
    e = __builtin_fma(-x, r, 1.0);
    r = __builtin_fma(r, e, r);
    return r == r ? r : r0;
}

// out[0] f32 mismatches, out[1] f64 mismatches, out[2..] per-exponent f32 mismatch counts (256),
// out[258..] per-exponent f64 mismatch counts (256)
__global__ void k_check(unsigned long long* out, uint32_t* samples) {
    const uint64_t n = 1ull << 32;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long bad32 = 0, bad64 = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t u = (uint32_t)i;
        const float x = __uint_as_float(u);
        const float a = rcp_f32(x), b = 1.0f / x;
        const bool ok32 = __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
        const double c = rcp_f64(x), d = 1.0 / (double)x;
        const bool ok64 = __double_as_longlong(c) == __double_as_longlong(d) || (c != c && d != d);
        const int ex = (int)((u >> 23) & 0xff);
        if (!ok32) {
            ++bad32;
            atomicAdd(&out[2 + ex], 1ull);
            if (samples[ex] == 0u) samples[ex] = u;
        }
        if (!ok64) {
            ++bad64;
            atomicAdd(&out[258 + ex], 1ull);
            if (samples[256 + ex] == 0u) samples[256 + ex] = u;
        }
    }
    if (bad32) atomicAdd(&out[0], bad32);
    if (bad64) atomicAdd(&out[1], bad64);
}

int main() {
    unsigned long long* d_out;
    uint32_t* d_s;
    if (hipMalloc(&d_out, 514 * sizeof(unsigned long long)) != hipSuccess) return 1;
    if (hipMalloc(&d_s, 512 * sizeof(uint32_t)) != hipSuccess) return 1;
    (void)hipMemset(d_out, 0, 514 * sizeof(unsigned long long));
    (void)hipMemset(d_s, 0, 512 * sizeof(uint32_t));
    hipLaunchKernelGGL(k_check, dim3(8192), dim3(256), 0, 0, d_out, d_s);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    unsigned long long out[514];
    uint32_t s[512];
    (void)hipMemcpy(out, d_out, sizeof(out), hipMemcpyDeviceToHost);
    (void)hipMemcpy(s, d_s, sizeof(s), hipMemcpyDeviceToHost);
    printf("{\"f32_mismatches\": %llu, \"f64_mismatches\": %llu, \"f32_by_exponent\": {", out[0], out[1]);
    bool first = true;
    for (int e = 0; e < 256; ++e)
        if (out[2 + e]) { printf("%s\"%d\": [%llu, \"0x%08x\"]", first ? "" : ", ", e, out[2 + e], s[e]); first = false; }
    printf("}, \"f64_by_exponent\": {");
    first = true;
    for (int e = 0; e < 256; ++e)
        if (out[258 + e]) { printf("%s\"%d\": [%llu, \"0x%08x\"]", first ? "" : ", ", e, out[258 + e], s[256 + e]); first = false; }
    printf("}}\n");
    return 0;
}
