// Schedules of the MSV row (S = 88 states per lane, 22 float4 chunks) with the kernel's real data
// dependencies, emissions held in registers (no LDS), to compare VALU orderings:
//   C: per chunk [4 max][4 add][2 max3]            (what the compiler emits)
//   D: per chunk [max3 max add max add max3 max add max add] (max3s fed by the previous chunk)
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 400;

template <int SCHED>
__global__ __launch_bounds__(256) void k(float* out, float bt0) {
    float M[88];
#pragma unroll
    for (int j = 0; j < 88; ++j) M[j] = -1.0f * j - threadIdx.x * 0.001f;
    const float e0 = 0.25f, e1 = -0.5f, e2 = 0.125f, e3 = -0.75f;
    float Bt = bt0;
    float acc = 0.f;
    for (int it = 0; it < ITERS; ++it) {
        float p0 = -1e30f, p1 = -1e30f;
#pragma unroll
        for (int c = 21; c >= 0; --c) {
            const int k = 4 * c;
            float& m0 = M[k];
            float& m1 = M[k + 1];
            float& m2 = M[k + 2];
            float& m3 = M[k + 3];
            const float prev = c > 0 ? M[k - 1] : -1e30f;
            if constexpr (SCHED == 0) {
                asm volatile(
                    "v_max_f32 %0, %1, %7\n\t"
                    "v_max_f32 %1, %2, %7\n\t"
                    "v_max_f32 %2, %3, %7\n\t"
                    "v_max_f32 %3, %6, %7\n\t"
                    "v_add_f32 %0, %8, %0\n\t"
                    "v_add_f32 %1, %9, %1\n\t"
                    "v_add_f32 %2, %10, %2\n\t"
                    "v_add_f32 %3, %11, %3\n\t"
                    "v_max3_f32 %4, %4, %0, %1\n\t"
                    "v_max3_f32 %5, %5, %2, %3"
                    : "+v"(m3), "+v"(m2), "+v"(m1), "+v"(m0), "+v"(p0), "+v"(p1)
                    : "v"(prev), "v"(Bt), "v"(e3), "v"(e2), "v"(e1), "v"(e0));
            } else {
                asm volatile(
                    "v_max_f32 %0, %1, %7\n\t"
                    "v_max_f32 %1, %2, %7\n\t"
                    "v_add_f32 %0, %8, %0\n\t"
                    "v_max_f32 %2, %3, %7\n\t"
                    "v_add_f32 %1, %9, %1\n\t"
                    "v_max_f32 %3, %6, %7\n\t"
                    "v_add_f32 %2, %10, %2\n\t"
                    "v_max3_f32 %4, %4, %0, %1\n\t"
                    "v_add_f32 %3, %11, %3\n\t"
                    "v_max3_f32 %5, %5, %2, %3"
                    : "+v"(m3), "+v"(m2), "+v"(m1), "+v"(m0), "+v"(p0), "+v"(p1)
                    : "v"(prev), "v"(Bt), "v"(e3), "v"(e2), "v"(e1), "v"(e0));
            }
        }
        Bt = Bt + 0.001f * (p0 > p1);
        acc += p0;
    }
    float s = acc;
#pragma unroll
    for (int j = 0; j < 88; ++j) s += M[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
void run(const char* name, K kern, float* d) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(256 * 4), dim3(256), 0, 0, d, -3.f);  // 4 blocks x 4 waves per CU
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(256 * 4), dim3(256), 0, 0, d, -3.f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double cells = 5.0 * 256 * 4 * 256 * double(ITERS) * 88;
    std::printf("{\"sched\": \"%s\", \"ms\": %.4f, \"cells_per_ns_per_simd\": %.3f}\n", name, ms,
                cells / (ms * 1e6) / 1024.0);
}

int main() {
    float* d;
    (void)hipMalloc(&d, sizeof(float) * 256 * 4 * 256 * 2);
    for (int r = 0; r < 2; ++r) {
        run("C_max4_add4_max3x2", k<0>, d);
        run("D_max3_interleaved", k<1>, d);
    }
    return 0;
}
