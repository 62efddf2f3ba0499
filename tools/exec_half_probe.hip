// exec_half_probe.hip — does a wave64 VALU instruction on gfx950 (two 32-lane passes per
// instruction) cost less when one half of the exec mask is empty?  Every wave runs the same
// f32 FMA stream (8 independent chains) on the lanes a mask selects; the kernel time for
// masks {all 64, lanes 0-31, lanes 32-63, even lanes, 16 lanes, 1 lane} tells whether the
// hardware skips an empty half.  Used to decide whether regrouping a wave's working lanes
// into one half pays.
//   hipcc --offload-arch=gfx950 -O3 -o build/exec_half_probe tools/exec_half_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

// clk[block] = shader-clock MHz over the kernel (s_memtime / s_memrealtime at 100 MHz), lane 0
// of wave 0 of each block: tells a clock drop (DVFS) from an issue cost
__global__ void __launch_bounds__(256) k_probe(float* out, uint64_t mask, int iters, float* clk) {
    const int lane = threadIdx.x & 63;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    float a0 = lane, a1 = lane + 1, a2 = lane + 2, a3 = lane + 3, a4 = lane + 4, a5 = lane + 5, a6 = lane + 6,
          a7 = lane + 7;
    if ((mask >> lane) & 1ull) {
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                a0 = __builtin_fmaf(a0, 1.0001f, 0.5f); a1 = __builtin_fmaf(a1, 1.0001f, 0.5f);
                a2 = __builtin_fmaf(a2, 1.0001f, 0.5f); a3 = __builtin_fmaf(a3, 1.0001f, 0.5f);
                a4 = __builtin_fmaf(a4, 1.0001f, 0.5f); a5 = __builtin_fmaf(a5, 1.0001f, 0.5f);
                a6 = __builtin_fmaf(a6, 1.0001f, 0.5f); a7 = __builtin_fmaf(a7, 1.0001f, 0.5f);
            }
        }
    }
    const float s = ((a0 + a1) + (a2 + a3)) + ((a4 + a5) + (a6 + a7));
    if (s == 1.2345f) out[0] = s;
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && clk) clk[blockIdx.x] = (float)((double)(t1 - t0) / (double)(r1 - r0) * 100.0);
}

// the same with f64 FMAs (the integrator's exact sequences are partly double precision)
__global__ void __launch_bounds__(256) k_probe64(double* out, uint64_t mask, int iters) {
    const int lane = threadIdx.x & 63;
    double a0 = lane, a1 = lane + 1, a2 = lane + 2, a3 = lane + 3;
    if ((mask >> lane) & 1ull) {
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 32; ++k) {
                a0 = __builtin_fma(a0, 1.0001, 0.5); a1 = __builtin_fma(a1, 1.0001, 0.5);
                a2 = __builtin_fma(a2, 1.0001, 0.5); a3 = __builtin_fma(a3, 1.0001, 0.5);
            }
        }
    }
    const double s = (a0 + a1) + (a2 + a3);
    if (s == 1.2345) out[0] = s;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* out;
    hipMalloc(&out, 64);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const struct { const char* name; uint64_t m; } masks[] = {
        {"all 64", ~0ull}, {"lanes 0-31", 0xffffffffull}, {"lanes 32-63", 0xffffffff00000000ull},
        {"even lanes", 0x5555555555555555ull}, {"lanes 0-15", 0xffffull}, {"lanes 48-63", 0xffff000000000000ull},
        {"every 4th (16)", 0x1111111111111111ull}, {"0-7 + 32-39", 0x000000ff000000ffull},
        {"lanes 0-14", 0x7fffull}, {"lanes 0-11", 0xfffull}, {"lanes 0-8", 0x1ffull}, {"lanes 0-7", 0xffull},
        {"lanes 8-15", 0xff00ull}, {"every 8th (8)", 0x0101010101010101ull},
        {"lanes 0-3", 0xfull}, {"lanes 0-1", 0x3ull}, {"lane 0", 1ull}, {"lanes 0,32", 0x100000001ull}};
    float* clk;
    hipMalloc(&clk, 4 * cus * sizeof(float));
    float* hclk = (float*)malloc(4 * cus * sizeof(float));
    const int iters = 4096;
    for (int wps = 1; wps <= 1; wps *= 4) {   // waves per SIMD: 1 (issue of one wave) and 4 (throughput)
        for (int f64 = 0; f64 < 1; ++f64) {
            for (const auto& m : masks) {
                const dim3 grid(cus * wps), block(256);
                if (f64) hipLaunchKernelGGL(k_probe64, grid, block, 0, 0, (double*)out, m.m, 8);
                else hipLaunchKernelGGL(k_probe, grid, block, 0, 0, out, m.m, 8, (float*)nullptr);
                hipEventRecord(a);
                if (f64) hipLaunchKernelGGL(k_probe64, grid, block, 0, 0, (double*)out, m.m, iters);
                else hipLaunchKernelGGL(k_probe, grid, block, 0, 0, out, m.m, iters, clk);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms = 0;
                hipEventElapsedTime(&ms, a, b);
                const double instrs = (double)iters * 128.0;   // FMAs per wave
                const double cyc = ms * 1e-3 * 2.4e9 / (instrs * wps);
                float mhz = 0;
                if (!f64) {
                    hipMemcpy(hclk, clk, grid.x * sizeof(float), hipMemcpyDeviceToHost);
                    double sum = 0;
                    for (unsigned i = 0; i < grid.x; ++i) sum += hclk[i];
                    mhz = (float)(sum / grid.x);
                }
                printf("%s waves/SIMD %d  %-12s %8.3f ms  %.2f cycles per wave-instruction per SIMD (at 2.4 GHz)  "
                       "in-kernel clock %.0f MHz\n", f64 ? "f64" : "f32", wps, m.name, ms, cyc, mhz);
            }
        }
    }
    return 0;
}
