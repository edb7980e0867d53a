// msv_kernel.hip -- the MSV hot path as ONE fused CDNA4 (gfx950) kernel per batch.
//
// Replaces MSV_HMM::parallel_run_on_sequence (algorithms/MSV_HMM.cpp:269-430) and its six
// OpenCL kernels (algorithms/MSV_kernels.cl:1-65, MSV_spec_kernels.cl:1-50): the reference
// launches 9-14 kernels PER RESIDUE for ONE sequence; here one persistent launch scores a whole
// batch of sequences against one profile, with every DP row kept on-chip.
//
// Recurrence (bit-exact restatement of MSV_HMM::run_on_sequence, MSV_HMM.cpp:100-112), for a
// residue r at row i:
//     Bt   = B' + tr_B_Mk
//     M_j  = e[r][j] + max(M'_{j-1}, Bt)          j = 1..LENG, M'_0 = -inf
//     E    = max_j M_j
//     J    = max(J' + loop, E + tEJ);  C = max(C' + loop, E + tEC)
//     N    = N' + loop;                B = max(N + move, J + move) == max(N, J) + move
// score = C_L + move.  Only IEEE adds and maxes: max is exact and fl() is monotone, so
// max(N+move, J+move) == fl(max(N,J) + move) bit for bit; no multiply exists, so no contraction.
//
// Mapping (MI355X-first, not a translation of the OpenCL NDRange-per-residue):
//   * A "group" of G lanes (G = 16, 32 or 64; 4/8 for small profiles) owns ONE sequence; lane gl holds the S consecutive
//     match states gl*S+1 .. gl*S+S of the DP row in VGPRs (float M[S]).  A 64-lane wave runs
//     64/G independent sequences.
//   * The j-1 neighbour crosses a lane boundary once per row: one DPP row_shr:1 (+ row_bcast:15
//     for G=32) moves M[S-1] to the next lane; lane 0 of a group reads M_0 = -inf.
//   * E: per-lane max3 tree, then a DPP butterfly (quad_perm, row_half_mirror, row_mirror) and a
//     v_permlane16_swap for G=32 -- no LDS, no barrier.
//   * The 20 x (G*S) fp32 emission table (+1 poison row of +inf for codes >= 20) lives in LDS,
//     laid out [residue][chunk][lane] float4 so every ds_read_b128 of a group is contiguous.
//     One workgroup per CU shares the table across all its waves.  Profiles whose table does not
//     fit the 160 KiB LDS (LENG > ~1920) use the SPLIT layout: each lane's first SA states have all
//     20 rows in LDS, its last S - SA states come from a lane-contiguous global table (L2), read one
//     row ahead as float4; beyond 3072 states the G = 64 row-class layout serves whole rows from LDS
//     or L2 behind a wave-uniform branch.
//   * Persistent grid: every group dequeues sequences from a device counter (prefetched one
//     sequence ahead, one atomic per sequence), so long and short sequences load-balance with no
//     host scheduling; a group that reaches the end of its sequence writes the score and starts
//     the next one in place.
//   * The residue stream is read one byte per row per group (global_load_ubyte, L1/L2-served,
//     1-6 rows of prefetch into rotating slots, by row length); the per-length transition
//     constants come from a host-computed table (host logf, so scores never depend on a device
//     logf).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <type_traits>
#include <utility>
#include <vector>

#include "msv_kernel_impl.h"

namespace msvk {

// ------------------------------------------------------------------------------------------------
// Longest-first dequeue order: a device counting sort on sequence length (lengths >= nbins-1 share
// the first bin).  Two small launches, histograms privatised in LDS so global atomics are one
// per (block, non-empty bin):  count (+ scan by the last block to finish) -> place.  Order inside a
// bin is arbitrary (it never changes a score: every score is written to its own sequence's slot).
// The scratch is [hist | cursor | ticket]: the scan writes the cursors and zeroes the histogram and
// the ticket for the next sort, so no memset launch precedes a sort (the caller zeroes a fresh or
// failed scratch once).  (A separate one-block scan launch cost ~5 us of launch latency per sort.)
// ------------------------------------------------------------------------------------------------
constexpr int kOrderThreads = 1024;

__device__ __forceinline__ uint32_t length_bin(const uint64_t* __restrict__ offsets, uint64_t s, uint32_t nbins) {
    const uint64_t L = offsets[s + 1] - offsets[s];
    return nbins - 1 - static_cast<uint32_t>(L >= nbins - 1 ? nbins - 1 : L);  // descending length
}

// Exclusive prefix sum of one value per thread over the block (kOrderThreads threads): a shuffle scan
// inside each wave, the 16 wave totals scanned by wave 0, two barriers (a Hillis-Steele scan over the
// block took 10 steps of two barriers each, ~5 us of a sort).  part: >= 16 words of LDS.
__device__ __forceinline__ uint32_t block_exclusive_sum(uint32_t v, uint32_t* part) {
    constexpr uint32_t kWaves = kOrderThreads / 64;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= static_cast<uint32_t>(d)) x += y;
    }
    if (lane == 63) part[w] = x;
    __syncthreads();
    if (w == 0) {
        uint32_t t = lane < kWaves ? part[lane] : 0u;
#pragma unroll
        for (int d = 1; d < static_cast<int>(kWaves); d <<= 1) {
            const uint32_t y = __shfl_up(t, d, 64);
            if (lane >= static_cast<uint32_t>(d)) t += y;
        }
        if (lane < kWaves) part[lane] = t;
    }
    __syncthreads();
    return (w ? part[w - 1] : 0u) + x - v;
}

// Exclusive scan of hist[nbins] into cursor[nbins], hist zeroed (one block, nbins <= 4 * kOrderThreads;
// part: 16 words of LDS).  hist is read with device-scope loads: the other blocks' counts arrived by
// atomics at L2.  Self-checking: the counts must total n (every sequence counted once).  The other
// blocks drained their count atomics (vmcnt) before taking their tickets, so the first read sees them
// all on gfx950 (MI355X_MICROARCH.md, inter-workgroup visibility); the HIP memory model does not
// promise it without a release/acquire pair, so a short total is re-read after an agent-scope acquire
// (the rare path pays the fence, the common one nothing), a bounded number of times.  If the counts
// never total n the sort is poisoned (*bad = 1): order_place_kernel then writes an out-of-range index
// into every slot, which the MSV kernel reports (kErrBadOrder) instead of scoring a wrong permutation.
__device__ __forceinline__ void scan_bins(uint32_t* __restrict__ hist, uint32_t* __restrict__ cursor, uint32_t nbins,
                                          uint32_t n, uint32_t* __restrict__ bad, uint32_t* part) {
    constexpr uint32_t kWaves = kOrderThreads / 64;
    const uint32_t t = threadIdx.x;
    uint32_t v[4], run = 0;
    bool ok = false;
    for (int attempt = 0; attempt < 64 && !ok; ++attempt) {
        if (attempt > 0) {
            __builtin_amdgcn_s_sleep(8);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        uint32_t sum = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t i = 4 * t + q;
            v[q] = i < nbins ? __hip_atomic_load(&hist[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
            sum += v[q];
        }
        run = block_exclusive_sum(sum, part);
        ok = part[kWaves - 1] == n;  // the block total (inclusive scan of the wave totals)
        __syncthreads();             // part is rewritten by the next attempt
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t i = 4 * t + q;
        if (i < nbins) {
            hist[i] = 0u;
            cursor[i] = run;
        }
        run += v[q];
    }
    if (t == 0) *bad = ok ? 0u : 1u;
}

// scratch = [hist | cursor | ticket | bad]; the last block to add its counts runs the scan, and no
// block waits for another.  The hand-off needs no fence in the common case: the counts are agent-scope
// atomics (performed past the XCD's L2), every wave drains them (vmcnt) before the block's ticket add,
// and the block whose add returns the last ticket reads them with sc1 loads after a barrier, checking
// that they total n (scan_bins).  A __threadfence() in every block (L2 write-back + invalidate) made
// this launch 57 us instead of 5.
__global__ __launch_bounds__(kOrderThreads) void order_count_kernel(const uint64_t* __restrict__ offsets, uint64_t n,
                                                                    uint64_t chunk, uint32_t* __restrict__ scratch,
                                                                    uint32_t nbins) {
    extern __shared__ uint32_t lh[];  // nbins words: block counts, then the scan partials (last block)
    __shared__ uint32_t ticket;
    uint32_t* const hist = scratch;
    for (uint32_t i = threadIdx.x; i < nbins; i += blockDim.x) lh[i] = 0;
    __syncthreads();
    const uint64_t lo = blockIdx.x * chunk, hi = min(n, lo + chunk);
    for (uint64_t s = lo + threadIdx.x; s < hi; s += blockDim.x) atomicAdd(&lh[length_bin(offsets, s, nbins)], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nbins; i += blockDim.x)
        if (lh[i]) atomicAdd(&hist[i], lh[i]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's count atomics have completed
    __syncthreads();
    if (threadIdx.x == 0) ticket = atomicAdd(scratch + 2 * nbins, 1u);
    __syncthreads();
    if (ticket != gridDim.x - 1) return;
    scan_bins(hist, scratch + nbins, nbins, static_cast<uint32_t>(n), scratch + 2 * nbins + 1, lh);
    if (threadIdx.x == 0) scratch[2 * nbins] = 0u;
}

__global__ __launch_bounds__(kOrderThreads) void order_place_kernel(const uint64_t* __restrict__ offsets, uint64_t n,
                                                                    uint64_t chunk, uint32_t* __restrict__ cursor,
                                                                    uint32_t nbins, uint32_t* __restrict__ order) {
    extern __shared__ uint32_t lh[];  // [0, nbins): block counts, then block cursors
    const uint64_t lo = blockIdx.x * chunk, hi = min(n, lo + chunk);
    if (cursor[nbins + 1]) {  // the count kernel's scan found a short total: poison every slot (scan_bins)
        for (uint64_t s = lo + threadIdx.x; s < hi; s += blockDim.x) order[s] = 0xFFFFFFFFu;
        return;
    }
    for (uint32_t i = threadIdx.x; i < nbins; i += blockDim.x) lh[i] = 0;
    __syncthreads();
    for (uint64_t s = lo + threadIdx.x; s < hi; s += blockDim.x) atomicAdd(&lh[length_bin(offsets, s, nbins)], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nbins; i += blockDim.x)
        if (lh[i]) lh[i] = atomicAdd(&cursor[i], lh[i]);  // reserve this block's range of bin i
    __syncthreads();
    for (uint64_t s = lo + threadIdx.x; s < hi; s += blockDim.x) {
        const uint32_t slot = atomicAdd(&lh[length_bin(offsets, s, nbins)], 1u);
        if (slot < n) order[slot] = static_cast<uint32_t>(s);  // (always, given the checked counts)
    }
}

// ------------------------------------------------------------------------------------------------
// MSV filter P-values (msv.h): one thread per sequence, HBM-bound elementwise
// (12 B read + 8 B written per sequence).  Same float/double steps as msv_stats.cpp's host path.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void msv_pvalues_kernel(const float* __restrict__ scores,
                                                          const uint64_t* __restrict__ offsets, uint64_t n, float mu,
                                                          float lambda, double* __restrict__ out) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) out[i] = msv_pvalue_of(scores[i], offsets[i + 1] - offsets[i], mu, lambda);
}

hipError_t launch_pvalues(const float* scores, const uint64_t* offsets, uint64_t n, float mu, float lambda,
                          double* pvalues, hipStream_t stream) {
    const uint64_t blocks = (n + 255) / 256;
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(msv_pvalues_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, stream, scores, offsets,
                       n, mu, lambda, pvalues);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Variant table: every compiled instantiation, in msv_variants_0.inc .. msv_variants_7.inc order (each
// part is its own translation unit, msv_kernel_part.hip; gen_variants.py writes them).  The host picks
// the one whose G*S covers LENG with the least estimated cost (the analog of the reference's
// should_specialize, which bakes sizes into the OpenCL program with -D defines, MSV_HMM.cpp:322-337).
// ------------------------------------------------------------------------------------------------
#define MSV_PART_DECL(k) const Variant* variants_part_##k(int* count);
MSV_PART_DECL(0) MSV_PART_DECL(1) MSV_PART_DECL(2) MSV_PART_DECL(3)
MSV_PART_DECL(4) MSV_PART_DECL(5) MSV_PART_DECL(6) MSV_PART_DECL(7)
#undef MSV_PART_DECL

const Variant* variants(int* count) {
    static const std::vector<Variant> all = [] {
        std::vector<Variant> v;
        for (auto part : {variants_part_0, variants_part_1, variants_part_2, variants_part_3, variants_part_4,
                          variants_part_5, variants_part_6, variants_part_7}) {
            int n = 0;
            const Variant* p = part(&n);
            v.insert(v.end(), p, p + n);
        }
        return v;
    }();
    *count = static_cast<int>(all.size());
    return all.data();
}

hipError_t launch_variant(const Variant& v, dim3 grid, const KernelArgs& args, hipStream_t stream, hipEvent_t start,
                          hipEvent_t stop, bool host_residues, bool clock) {
    void* params[] = {const_cast<KernelArgs*>(&args)};
    const void* fn = host_residues && v.zc_fn ? v.zc_fn : v.fn;
    if (clock && v.clock_fn && !host_residues) fn = v.clock_fn;
    if (start || stop) return hipExtLaunchKernel(fn, grid, dim3(v.waves * 64), params, 0, stream, start, stop, 0);
    return hipLaunchKernel(fn, grid, dim3(v.waves * 64), params, 0, stream);
}

hipError_t launch_grid_variant(const Variant& v, const GridArgs& args, hipStream_t stream) {
    if (!v.grid_fn || args.profiles == 0 || args.profiles > kGridMaxProfiles || args.per_profile == 0)
        return hipErrorInvalidValue;
    void* params[] = {const_cast<GridArgs*>(&args)};
    return hipLaunchKernel(v.grid_fn, dim3(args.profiles * args.per_profile), dim3(v.waves * 64), params, 0, stream);
}

// Small batches (n <= kSmallOrderPer * kOrderThreads): the whole counting sort in ONE launch and one
// workgroup (histogram, scan and cursors in LDS, no memset), lengths held in registers between the
// passes.  Replaces 4 dependent launches (~17 us of launch latency) by one (~5 us).
constexpr int kSmallOrderPer = 16;

__global__ __launch_bounds__(kOrderThreads) void order_small_kernel(const uint64_t* __restrict__ offsets, uint32_t n,
                                                                    uint32_t nbins, uint32_t* __restrict__ order) {
    extern __shared__ uint32_t lh[];  // [nbins] counts -> cursors, [kOrderThreads] scan partials
    uint32_t* part = lh + nbins;
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < nbins; i += kOrderThreads) lh[i] = 0;
    uint32_t bin[kSmallOrderPer];
#pragma unroll
    for (int k = 0; k < kSmallOrderPer; ++k) {
        const uint32_t s = t + k * kOrderThreads;
        bin[k] = s < n ? length_bin(offsets, s, nbins) : 0xFFFFFFFFu;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSmallOrderPer; ++k)
        if (bin[k] != 0xFFFFFFFFu) atomicAdd(&lh[bin[k]], 1u);
    __syncthreads();
    // exclusive scan of lh[0..nbins): 4 consecutive bins per thread, block_exclusive_sum over threads
    uint32_t v[4], sum = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t i = 4 * t + q;
        v[q] = i < nbins ? lh[i] : 0u;
        sum += v[q];
    }
    uint32_t run = block_exclusive_sum(sum, part);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t i = 4 * t + q;
        if (i < nbins) lh[i] = run;
        run += v[q];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSmallOrderPer; ++k)
        if (bin[k] != 0xFFFFFFFFu) order[atomicAdd(&lh[bin[k]], 1u)] = t + k * kOrderThreads;
}

hipError_t launch_order(const uint64_t* offsets, uint64_t n, uint32_t* scratch_hist, uint32_t nbins, uint32_t* order,
                        hipStream_t stream) {
    if (nbins > 4 * kOrderThreads || nbins < kOrderThreads) return hipErrorInvalidValue;
    if (n <= static_cast<uint64_t>(kSmallOrderPer) * kOrderThreads) {
        const size_t lds = (nbins + kOrderThreads) * sizeof(uint32_t);
        hipLaunchKernelGGL(order_small_kernel, dim3(1), dim3(kOrderThreads), lds, stream, offsets,
                           static_cast<uint32_t>(n), nbins, order);
        return hipGetLastError();
    }
    const uint64_t blocks = std::min<uint64_t>(256, (n + 511) / 512);
    const uint64_t chunk = (n + blocks - 1) / blocks;
    const size_t lds = nbins * sizeof(uint32_t);
    hipLaunchKernelGGL(order_count_kernel, dim3(blocks), dim3(kOrderThreads), lds, stream, offsets, n, chunk,
                       scratch_hist, nbins);
    hipLaunchKernelGGL(order_place_kernel, dim3(blocks), dim3(kOrderThreads), lds, stream, offsets, n, chunk,
                       scratch_hist + nbins, nbins, order);
    return hipGetLastError();
}

}  // namespace msvk
