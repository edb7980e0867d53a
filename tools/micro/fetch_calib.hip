// FETCH_SIZE calibration for the MSV kernel's narrow reads (gfx950).  MI355X_MICROARCH.md §HBM:
// FETCH_SIZE reports exactly 1/2 of the bytes of a wide coalesced streaming read; other access
// widths are uncalibrated.  Each kernel below reads a KNOWN number of bytes of a 400 MB buffer
// (past the 256 MiB Infinity Cache) exactly once, in one access pattern:
//   k_stream_f4   : 16 B/lane coalesced grid-stride read (the guide's calibrated case, factor 2)
//   k_ubyte_lane  : global_load_ubyte, every lane walks its own contiguous 400-byte segment
//   k_ubyte_group : global_load_ubyte, 16 lanes read the same byte and each 16-lane group walks
//                   its own 400-byte segment one byte per step -- the MSV kernel's residue stream
// Run under rocprofv3 --pmc FETCH_SIZE; tools/fetch_calib_summary.py divides the known bytes by
// FETCH_SIZE per dispatch.
// Build: hipcc --offload-arch=gfx950 -O3 -o fetch_calib fetch_calib.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

constexpr uint64_t kBytes = 400ull << 20;
constexpr int kSeg = 400;

__global__ __launch_bounds__(256) void k_stream_f4(const uint4* __restrict__ in, uint64_t n16, uint32_t* out) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += gridDim.x * 256ull) {
        const uint4 v = in[i];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void k_ubyte_lane(const uint8_t* __restrict__ in, uint64_t nseg, uint32_t* out) {
    const uint64_t t = blockIdx.x * 256ull + threadIdx.x;
    uint32_t acc = 0;
    if (t < nseg) {
        const uint8_t* p = in + t * kSeg;
        for (int k = 0; k < kSeg; ++k) acc += p[k];
    }
    out[t] = acc;
}

__global__ __launch_bounds__(256) void k_ubyte_group(const uint8_t* __restrict__ in, uint64_t nseg, uint32_t* out) {
    const uint64_t t = blockIdx.x * 256ull + threadIdx.x;
    const uint64_t g = t >> 4;  // 16-lane group
    uint32_t acc = 0;
    if (g < nseg) {
        const uint8_t* p = in + g * kSeg;
        for (int k = 0; k < kSeg; ++k) acc += p[k];  // same address in all 16 lanes of the group
    }
    out[t] = acc;
}

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
            return 1;                                                             \
        }                                                                         \
    } while (0)

int main() {
    uint8_t* d = nullptr;
    uint32_t* out = nullptr;
    const uint64_t nseg = kBytes / kSeg;
    const uint64_t threads = nseg * 16;  // k_ubyte_group has the most threads
    CHECK(hipMalloc(&d, kBytes));
    CHECK(hipMalloc(&out, threads * sizeof(uint32_t)));
    CHECK(hipMemset(d, 7, kBytes));
    CHECK(hipDeviceSynchronize());
    const uint64_t covered = nseg * kSeg;
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_stream_f4, dim3(256 * 8), dim3(256), 0, 0, reinterpret_cast<const uint4*>(d), kBytes / 16,
                           out);
        hipLaunchKernelGGL(k_ubyte_lane, dim3(static_cast<uint32_t>((nseg + 255) / 256)), dim3(256), 0, 0, d, nseg, out);
        hipLaunchKernelGGL(k_ubyte_group, dim3(static_cast<uint32_t>((threads + 255) / 256)), dim3(256), 0, 0, d, nseg,
                           out);
        CHECK(hipGetLastError());
    }
    CHECK(hipDeviceSynchronize());
    std::printf("{\"k_stream_f4\": %llu, \"k_ubyte_lane\": %llu, \"k_ubyte_group\": %llu}\n",
                static_cast<unsigned long long>(kBytes), static_cast<unsigned long long>(covered),
                static_cast<unsigned long long>(covered));
    CHECK(hipFree(d));
    CHECK(hipFree(out));
    return 0;
}
