// VALU issue-rate microbenchmark (gfx950): wave64 instructions per SIMD per clock for the
// instruction forms the MSV cell update can use.  Each lane runs NCH independent chains so a
// single wave is never dependency-bound; waves per SIMD is swept via the block size.
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_rate valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int ITERS = 2048;

__global__ void k_A_maxadd4_max3x2(float* out, float a, float b) {
    float x[12];
#pragma unroll
    for (int c = 0; c < 12; ++c) x[c] = threadIdx.x * 0.001f + c;
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[11]) : "v"(a), "v"(a));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < 12; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_B_interleave_max3(float* out, float a, float b) {
    float x[12];
#pragma unroll
    for (int c = 0; c < 12; ++c) x[c] = threadIdx.x * 0.001f + c;
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[11]) : "v"(a), "v"(a));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < 12; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_C_max4_add4_max3x2(float* out, float a, float b) {
    float x[12];
#pragma unroll
    for (int c = 0; c < 12; ++c) x[c] = threadIdx.x * 0.001f + c;
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[11]) : "v"(a), "v"(a));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < 12; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_D_max3_first(float* out, float a, float b) {
    float x[12];
#pragma unroll
    for (int c = 0; c < 12; ++c) x[c] = threadIdx.x * 0.001f + c;
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[11]) : "v"(a), "v"(a));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < 12; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_E_add_max_pairs(float* out, float a, float b) {
    float x[12];
#pragma unroll
    for (int c = 0; c < 12; ++c) x[c] = threadIdx.x * 0.001f + c;
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[11]) : "v"(a), "v"(a));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < 12; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_F_only_max6(float* out, float a, float b) {
    float x[12];
#pragma unroll
    for (int c = 0; c < 12; ++c) x[c] = threadIdx.x * 0.001f + c;
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[11]) : "v"(a), "v"(a));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < 12; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_G_max6_add2(float* out, float a, float b) {
    float x[12];
#pragma unroll
    for (int c = 0; c < 12; ++c) x[c] = threadIdx.x * 0.001f + c;
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[11]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[0]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[1]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[2]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[3]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[4]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[5]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[6]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[7]) : "v"(a), "v"(a));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[8]) : "v"(a), "v"(a));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[9]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[10]) : "v"(a), "v"(a));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[11]) : "v"(a), "v"(a));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < 12; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
void run(const char* name, K kern, int waves_per_simd, float* d, double instr_per_iter, double cells_per_iter) {
    int block = 64 * 4 * waves_per_simd;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(256), dim3(block), 0, 0, d, 1.f, 2.f);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(256), dim3(block), 0, 0, d, 1.f, 2.f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    double ns = ms * 1e6;
    double instr = 5.0 * waves_per_simd * ITERS * instr_per_iter;
    std::printf("{\"mix\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"ns_per_wave_instr_per_simd\": %.4f, \"cells_per_ns_per_simd\": %.3f}\n",
                name, waves_per_simd, ms, ns / instr, cells_per_iter > 0 ? 5.0 * waves_per_simd * ITERS * cells_per_iter * 64 / ns : 0.0);
}
int main() {
    float* d;
    (void)hipMalloc(&d, sizeof(float) * 256 * 64 * 16);
    for (int w : {4}) {
        run("A_maxadd4_max3x2", k_A_maxadd4_max3x2, w, d, 60, 24);
        run("B_interleave_max3", k_B_interleave_max3, w, d, 60, 24);
        run("C_max4_add4_max3x2", k_C_max4_add4_max3x2, w, d, 60, 24);
        run("D_max3_first", k_D_max3_first, w, d, 60, 24);
        run("E_add_max_pairs", k_E_add_max_pairs, w, d, 60, 24);
        run("F_only_max6", k_F_only_max6, w, d, 36, 0);
        run("G_max6_add2", k_G_max6_add2, w, d, 48, 0);
    }
    return 0;
}
