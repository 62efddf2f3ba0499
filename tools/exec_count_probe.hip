// exec_count_probe.hip — cost of a wave64 VALU instruction on gfx950 as a function of how many
// lanes are active.  For each instruction kind, every wave runs the same stream of CHAINS
// independent dependency chains on the lanes of a mask (popcount 1 .. 64, contiguous from lane
// 0); the in-kernel cycle count (s_memtime) per instruction is printed.  tools/exec_half_probe
// found instructions with few active lanes to be several times slower; this maps the cliff.
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -o build/exec_count_probe tools/exec_count_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

enum Op { FMA32, ADD32, FMA64, ADDU32, PKFMA, NOPS };
static const char* kOpName[] = {"v_fma_f32", "v_add_f32", "v_fma_f64", "v_add_u32", "v_pk_fma_f32"};

typedef float f2 __attribute__((ext_vector_type(2)));

template <int OP, int CHAINS>
__global__ void __launch_bounds__(1024) k_op(uint64_t mask, int iters, unsigned long long* cyc, float* sink, float mul) {
    const int lane = threadIdx.x & 63;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    float f[CHAINS];
    double d[CHAINS];
    uint32_t u[CHAINS];
    f2 p[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
        f[c] = (mul > 1.0f ? (float)lane : 1.0f) + c;
        d[c] = 1.0 + c;
        u[c] = lane + c;
        p[c] = f2{1.0f + c, 2.0f + c};
    }
    if ((mask >> lane) & 1ull) {
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
#pragma unroll
                for (int c = 0; c < CHAINS; ++c) {
                    if (OP == FMA32) f[c] = __builtin_fmaf(f[c], mul, 0.5f);
                    if (OP == ADD32) f[c] = f[c] + 0.5f;
                    if (OP == FMA64) d[c] = __builtin_fma(d[c], 0.9999, 0.5);
                    if (OP == ADDU32) u[c] = u[c] + 0x9e3779b9u;
                    if (OP == PKFMA) p[c] = __builtin_elementwise_fma(p[c], f2{0.9999f, 0.9999f}, f2{0.5f, 0.5f});
                }
            }
        }
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += f[c] + (float)d[c] + (float)u[c] + p[c].x + p[c].y;
    if (s == 1.2345f) sink[0] = s;
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

static int g_block = 64;
static float g_mul = 0.9999f;
template <int OP, int CHAINS>
static double run(uint64_t mask, int cus, unsigned long long* dcyc, float* sink) {
    const int iters = 2048;
    hipLaunchKernelGGL((k_op<OP, CHAINS>), dim3(cus), dim3(g_block), 0, 0, mask, iters, dcyc, sink, g_mul);
    hipDeviceSynchronize();
    static unsigned long long h[4096];
    hipMemcpy(h, dcyc, cus * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < cus; ++i) s += (double)h[i];
    return s / cus / ((double)iters * 8 * CHAINS);
}

template <int OP>
static void sweep(int cus, unsigned long long* dcyc, float* sink) {
    const int counts[] = {64, 48, 33, 32, 24, 17, 16, 12, 9, 8, 4, 1};
    printf("%-13s", kOpName[OP]);
    for (int n : counts) printf(" %6d", n);
    printf("   (active lanes; cycles per wave-instruction, one wave per CU)\n");
    for (int chains : {1, 8}) {
        printf("  chains %-4d", chains);
        for (int n : counts) {
            const uint64_t m = n == 64 ? ~0ull : ((1ull << n) - 1);
            const double c = chains == 1 ? run<OP, 1>(m, cus, dcyc, sink) : run<OP, 8>(m, cus, dcyc, sink);
            printf(" %6.2f", c);
        }
        printf("\n");
    }
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned long long* dcyc;
    float* sink;
    hipMalloc(&dcyc, 4096 * sizeof(unsigned long long));
    hipMalloc(&sink, 64);
    for (int block : {64, 128, 256, 1024}) {
        for (float mul : {0.9999f, 1.0001f}) {
            g_block = block;
            g_mul = mul;
            printf("== %d waves per CU, fma multiplier %.4f (1.0001: values start at the lane index and grow)\n",
                   block / 64, mul);
            sweep<FMA32>(cus, dcyc, sink);
        }
    }
    g_block = 256;
    g_mul = 0.9999f;
    printf("== 4 waves per CU\n");
    sweep<ADD32>(cus, dcyc, sink);
    sweep<FMA64>(cus, dcyc, sink);
    sweep<PKFMA>(cus, dcyc, sink);
    return 0;
}
