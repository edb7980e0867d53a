// VALU issue-rate microbenchmark (gfx950): wave64 instructions per SIMD per clock for the
// instruction forms the MSV cell update can use.  Each lane runs NCH independent chains so a
// single wave is never dependency-bound; waves per SIMD is swept via the block size.
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_rate valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int NCH = 16;
constexpr int ITERS = 2048;

__global__ void k_v_add_f32(float* out, float a, float b) {
    float x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_v_max_f32(float* out, float a, float b) {
    float x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_v_min_f32(float* out, float a, float b) {
    float x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_min_f32 %0, %0, %1" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_min_f32 %0, %0, %1" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_min_f32 %0, %0, %1" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_min_f32 %0, %0, %1" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_min_f32 %0, %0, %1" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_min_f32 %0, %0, %1" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_min_f32 %0, %0, %1" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_min_f32 %0, %0, %1" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_min_f32 %0, %0, %1" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_min_f32 %0, %0, %1" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_min_f32 %0, %0, %1" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_min_f32 %0, %0, %1" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_min_f32 %0, %0, %1" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_min_f32 %0, %0, %1" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_min_f32 %0, %0, %1" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_min_f32 %0, %0, %1" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_v_max3_f32(float* out, float a, float b) {
    float x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_v_maximum3_f32(float* out, float a, float b) {
    float x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_maximum3_f32 %0, %0, %1, %2" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_v_med3_f32(float* out, float a, float b) {
    float x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_v_max_i32(float* out, float a, float b) {
    float x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_v_max3_i32(float* out, float a, float b) {
    float x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_v_add_u32(float* out, float a, float b) {
    float x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_v_xor_b32(float* out, float a, float b) {
    float x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_v_cndmask_b32(float* out, float a, float b) {
    float x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_v_sub_f32(float* out, float a, float b) {
    float x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_sub_f32 %0, %0, %1" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_sub_f32 %0, %0, %1" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_sub_f32 %0, %0, %1" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_sub_f32 %0, %0, %1" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_sub_f32 %0, %0, %1" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_sub_f32 %0, %0, %1" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_sub_f32 %0, %0, %1" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_sub_f32 %0, %0, %1" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_sub_f32 %0, %0, %1" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_sub_f32 %0, %0, %1" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_sub_f32 %0, %0, %1" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_sub_f32 %0, %0, %1" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_sub_f32 %0, %0, %1" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_sub_f32 %0, %0, %1" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_sub_f32 %0, %0, %1" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_sub_f32 %0, %0, %1" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_v_mul_f32(float* out, float a, float b) {
    float x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_v_mov_b32(float* out, float a, float b) {
    float x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_mov_b32 %0, %1" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_mov_b32 %0, %1" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_mov_b32 %0, %1" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_mov_b32 %0, %1" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_mov_b32 %0, %1" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_mov_b32 %0, %1" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_mov_b32 %0, %1" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_mov_b32 %0, %1" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_mov_b32 %0, %1" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_mov_b32 %0, %1" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_mov_b32 %0, %1" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_mov_b32 %0, %1" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_mov_b32 %0, %1" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_mov_b32 %0, %1" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_mov_b32 %0, %1" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_mov_b32 %0, %1" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_v_max_f64(double* out, double a, double b) {
    double x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_max_f64 %0, %0, %1" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_max_f64 %0, %0, %1" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_max_f64 %0, %0, %1" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_max_f64 %0, %0, %1" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_max_f64 %0, %0, %1" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_max_f64 %0, %0, %1" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_max_f64 %0, %0, %1" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_max_f64 %0, %0, %1" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_max_f64 %0, %0, %1" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_max_f64 %0, %0, %1" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_max_f64 %0, %0, %1" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_max_f64 %0, %0, %1" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_max_f64 %0, %0, %1" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_max_f64 %0, %0, %1" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_max_f64 %0, %0, %1" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_max_f64 %0, %0, %1" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_v_add_f64(double* out, double a, double b) {
    double x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_max_add(float* out, float a, float b) {
    float x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_max_add_add(float* out, float a, float b) {
    float x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_max3_max_add(float* out, float a, float b) {
    float x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_max_max_add_add(float* out, float a, float b) {
    float x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_med3_add(float* out, float a, float b) {
    float x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_maxi32_add(float* out, float a, float b) {
    float x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_max_maxi32(float* out, float a, float b) {
    float x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_max_cnd(float* out, float a, float b) {
    float x[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) x[c] = threadIdx.x * 0.001f + c;
    asm volatile("s_mov_b64 vcc, -1");
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[0]) : "v"(a), "v"(b));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[1]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[2]) : "v"(a), "v"(b));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[3]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[4]) : "v"(a), "v"(b));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[5]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[6]) : "v"(a), "v"(b));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[7]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[8]) : "v"(a), "v"(b));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[9]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[10]) : "v"(a), "v"(b));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[11]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[12]) : "v"(a), "v"(b));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[13]) : "v"(a), "v"(b));
            asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[14]) : "v"(a), "v"(b));
            asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[15]) : "v"(a), "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename T, typename K>
void run(const char* name, K kern, int waves_per_simd, T* d) {
    int block = 64 * 4 * waves_per_simd;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(256), dim3(block), 0, 0, d, T(1), T(2));
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(256), dim3(block), 0, 0, d, T(1), T(2));
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    double instr = 5.0 * waves_per_simd * ITERS * NCH;
    std::printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"ns_per_wave_instr_per_simd\": %.4f}\n",
                name, waves_per_simd, ms, ms * 1e6 / instr);
}
int main() {
    double* d;
    (void)hipMalloc(&d, sizeof(double) * 256 * 64 * 16);
    for (int w : {1, 2, 4}) {
        run<float>("v_add_f32", k_v_add_f32, w, (float*)d);
        run<float>("v_max_f32", k_v_max_f32, w, (float*)d);
        run<float>("v_min_f32", k_v_min_f32, w, (float*)d);
        run<float>("v_max3_f32", k_v_max3_f32, w, (float*)d);
        run<float>("v_maximum3_f32", k_v_maximum3_f32, w, (float*)d);
        run<float>("v_med3_f32", k_v_med3_f32, w, (float*)d);
        run<float>("v_max_i32", k_v_max_i32, w, (float*)d);
        run<float>("v_max3_i32", k_v_max3_i32, w, (float*)d);
        run<float>("v_add_u32", k_v_add_u32, w, (float*)d);
        run<float>("v_xor_b32", k_v_xor_b32, w, (float*)d);
        run<float>("v_cndmask_b32", k_v_cndmask_b32, w, (float*)d);
        run<float>("v_sub_f32", k_v_sub_f32, w, (float*)d);
        run<float>("v_mul_f32", k_v_mul_f32, w, (float*)d);
        run<float>("v_mov_b32", k_v_mov_b32, w, (float*)d);
        run<double>("v_max_f64", k_v_max_f64, w, (double*)d);
        run<double>("v_add_f64", k_v_add_f64, w, (double*)d);
        run<float>("max+add", k_max_add, w, (float*)d);
        run<float>("max+add+add", k_max_add_add, w, (float*)d);
        run<float>("max3+max+add", k_max3_max_add, w, (float*)d);
        run<float>("max+max+add+add", k_max_max_add_add, w, (float*)d);
        run<float>("med3+add", k_med3_add, w, (float*)d);
        run<float>("maxi32+add", k_maxi32_add, w, (float*)d);
        run<float>("max+maxi32", k_max_maxi32, w, (float*)d);
        run<float>("max+cnd", k_max_cnd, w, (float*)d);
    }
    return 0;
}
