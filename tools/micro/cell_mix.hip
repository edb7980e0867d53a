// VALU issue-rate microbenchmark (gfx950): wave64 instructions per SIMD per clock for the
// instruction forms the MSV cell update can use.  Each lane runs NCH independent chains so a
// single wave is never dependency-bound; waves per SIMD is swept via the block size.
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_rate valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int ITERS = 2048;

__global__ void k_A(float* out, float a, float b) {
    float x[8];
    double y[8];
    double z = b;
#pragma unroll
    for (int c = 0; c < 8; ++c) { x[c] = threadIdx.x * 0.001f + c; y[c] = c; }
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[0]), "+v"(y[0]) : "v"(a), "v"(z));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[1]), "+v"(y[1]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[2]), "+v"(y[2]) : "v"(a), "v"(z));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[3]), "+v"(y[3]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[4]), "+v"(y[4]) : "v"(a), "v"(z));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[5]), "+v"(y[5]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[6]), "+v"(y[6]) : "v"(a), "v"(z));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[7]), "+v"(y[7]) : "v"(a), "v"(z));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[0]), "+v"(y[0]) : "v"(a), "v"(z));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[1]), "+v"(y[1]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[2]), "+v"(y[2]) : "v"(a), "v"(z));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[3]), "+v"(y[3]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[4]), "+v"(y[4]) : "v"(a), "v"(z));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[5]), "+v"(y[5]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[6]), "+v"(y[6]) : "v"(a), "v"(z));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[7]), "+v"(y[7]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[0]), "+v"(y[0]) : "v"(a), "v"(z));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[1]), "+v"(y[1]) : "v"(a), "v"(z));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[2]), "+v"(y[2]) : "v"(a), "v"(z));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[3]), "+v"(y[3]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[4]), "+v"(y[4]) : "v"(a), "v"(z));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[5]), "+v"(y[5]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[6]), "+v"(y[6]) : "v"(a), "v"(z));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[7]), "+v"(y[7]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[0]), "+v"(y[0]) : "v"(a), "v"(z));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[1]), "+v"(y[1]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[2]), "+v"(y[2]) : "v"(a), "v"(z));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[3]), "+v"(y[3]) : "v"(a), "v"(z));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[4]), "+v"(y[4]) : "v"(a), "v"(z));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[5]), "+v"(y[5]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[6]), "+v"(y[6]) : "v"(a), "v"(z));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[7]), "+v"(y[7]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[0]), "+v"(y[0]) : "v"(a), "v"(z));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[1]), "+v"(y[1]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[2]), "+v"(y[2]) : "v"(a), "v"(z));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[3]), "+v"(y[3]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[4]), "+v"(y[4]) : "v"(a), "v"(z));
            asm volatile("v_add_f32 %0, %0, %2" : "+v"(x[5]), "+v"(y[5]) : "v"(a), "v"(z));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[6]), "+v"(y[6]) : "v"(a), "v"(z));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[7]), "+v"(y[7]) : "v"(a), "v"(z));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) s += x[c] + (float)y[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_B(float* out, float a, float b) {
    float x[8];
    double y[8];
    double z = b;
#pragma unroll
    for (int c = 0; c < 8; ++c) { x[c] = threadIdx.x * 0.001f + c; y[c] = c; }
    for (int it = 0; it < ITERS; ++it) {
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[0]), "+v"(y[0]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[1]), "+v"(y[1]) : "v"(a), "v"(z));
            asm volatile("v_pk_add_f32 %1, %1, %3" : "+v"(x[2]), "+v"(y[2]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[3]), "+v"(y[3]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[4]), "+v"(y[4]) : "v"(a), "v"(z));
            asm volatile("v_pk_add_f32 %1, %1, %3" : "+v"(x[5]), "+v"(y[5]) : "v"(a), "v"(z));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[6]), "+v"(y[6]) : "v"(a), "v"(z));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[7]), "+v"(y[7]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[0]), "+v"(y[0]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[1]), "+v"(y[1]) : "v"(a), "v"(z));
            asm volatile("v_pk_add_f32 %1, %1, %3" : "+v"(x[2]), "+v"(y[2]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[3]), "+v"(y[3]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[4]), "+v"(y[4]) : "v"(a), "v"(z));
            asm volatile("v_pk_add_f32 %1, %1, %3" : "+v"(x[5]), "+v"(y[5]) : "v"(a), "v"(z));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[6]), "+v"(y[6]) : "v"(a), "v"(z));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[7]), "+v"(y[7]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[0]), "+v"(y[0]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[1]), "+v"(y[1]) : "v"(a), "v"(z));
            asm volatile("v_pk_add_f32 %1, %1, %3" : "+v"(x[2]), "+v"(y[2]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[3]), "+v"(y[3]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[4]), "+v"(y[4]) : "v"(a), "v"(z));
            asm volatile("v_pk_add_f32 %1, %1, %3" : "+v"(x[5]), "+v"(y[5]) : "v"(a), "v"(z));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[6]), "+v"(y[6]) : "v"(a), "v"(z));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[7]), "+v"(y[7]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[0]), "+v"(y[0]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[1]), "+v"(y[1]) : "v"(a), "v"(z));
            asm volatile("v_pk_add_f32 %1, %1, %3" : "+v"(x[2]), "+v"(y[2]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[3]), "+v"(y[3]) : "v"(a), "v"(z));
            asm volatile("v_max_f32 %0, %0, %2" : "+v"(x[4]), "+v"(y[4]) : "v"(a), "v"(z));
            asm volatile("v_pk_add_f32 %1, %1, %3" : "+v"(x[5]), "+v"(y[5]) : "v"(a), "v"(z));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[6]), "+v"(y[6]) : "v"(a), "v"(z));
            asm volatile("v_max3_f32 %0, %0, %2, %2" : "+v"(x[7]), "+v"(y[7]) : "v"(a), "v"(z));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) s += x[c] + (float)y[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
void run(const char* name, K kern, int waves_per_simd, float* d, int cells_per_iter) {
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
    double cells = 5.0 * waves_per_simd * ITERS * cells_per_iter * 64;
    std::printf("{\"mix\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"cells_per_ns_per_simd\": %.3f}\n",
                name, waves_per_simd, ms, cells / (ms * 1e6));
}
int main() {
    float* d;
    (void)hipMalloc(&d, sizeof(float) * 256 * 64 * 16);
    for (int w : {2, 3, 4}) {
        run("A_max_add_max3 (current)", k_A, w, d, 16);
        run("B_max_pkadd_max3", k_B, w, d, 16);
    }
    return 0;
}
