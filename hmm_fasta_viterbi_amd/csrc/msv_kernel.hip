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

#include "msv_kernel.h"

namespace msvk {

namespace {

template <int CTRL, int ROW_MASK = 0xF, int BANK_MASK = 0xF>
__device__ __forceinline__ float dpp(float old, float src) {
    // bound_ctrl = false: a lane whose DPP source is invalid keeps `old`.
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(src), CTRL, ROW_MASK,
                                                      BANK_MASK, false));
}

constexpr int DPP_QUAD_1032 = 0xB1;    // quad_perm:[1,0,3,2]
constexpr int DPP_QUAD_2301 = 0x4E;    // quad_perm:[2,3,0,1]
constexpr int DPP_ROW_SHR1 = 0x111;    // row_shr:1
constexpr int DPP_ROW_MIRROR = 0x140;  // row_mirror
constexpr int DPP_ROW_HMIRROR = 0x141; // row_half_mirror
constexpr int DPP_ROW_BCAST15 = 0x142; // row_bcast:15

// M_{j-1} for the first state of each lane: the last state of the previous lane of the same
// group; -inf (the dummy M0 column, MSV_HMM.cpp:86) for the first lane of a group.  `old` supplies
// the lanes the shift does not write: -inf there (G < 16: any value, the -inf is selected here).
// For G >= 16 the caller passes the previous result back in, so those lanes keep the -inf written
// once at start and no per-row -inf copy is needed.
template <int G>
__device__ __forceinline__ float shift_in(float last, float old) {
    if constexpr (G < 16) {
        static_assert(G == 4 || G == 8, "G must be 4, 8, 16, 32 or 64");
        const float v = dpp<DPP_ROW_SHR1>(old, last);
        return (threadIdx.x & (G - 1)) == 0 ? -__builtin_inff() : v;  // first lane of each group
    } else if constexpr (G == 16) {
        return dpp<DPP_ROW_SHR1>(old, last);
    } else if constexpr (G == 32) {
        // rows 1 and 3 first receive lane 15 of rows 0 and 2; row_shr:1 then fills every lane
        // except the first of each row, which keeps that broadcast (or -inf for rows 0 and 2).
        float v = dpp<DPP_ROW_BCAST15, 0xA>(old, last);
        return dpp<DPP_ROW_SHR1>(v, last);
    } else {
        static_assert(G == 64, "G must be 16, 32 or 64");
        float v = dpp<DPP_ROW_BCAST15, 0xE>(old, last);  // rows 1-3 get lane 15 of the row before
        return dpp<DPP_ROW_SHR1>(v, last);
    }
}

// In-row permutation (every source lane valid): lets the DPP combiner fold it into v_max_f32_dpp.
template <int CTRL>
__device__ __forceinline__ float dpp_perm(float src) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(src), CTRL, 0xF, 0xF, true));
}

// Lane q of each 16-lane DPP row, broadcast to the whole row (row_newbcast, gfx90a+).
template <int Q>
__device__ __forceinline__ uint32_t row_bcast_lane(uint32_t v) {
    static_assert(Q >= 0 && Q < 16, "row_newbcast lane");
    return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), 0x150 + Q, 0xF, 0xF, true));
}

// Max over the G lanes of a group, result in every lane of the group.
template <int G>
__device__ __forceinline__ float group_max(float x) {
    x = fmaxf(x, dpp_perm<DPP_QUAD_1032>(x));
    x = fmaxf(x, dpp_perm<DPP_QUAD_2301>(x));
    if constexpr (G >= 8) x = fmaxf(x, dpp_perm<DPP_ROW_HMIRROR>(x));
    if constexpr (G >= 16) x = fmaxf(x, dpp_perm<DPP_ROW_MIRROR>(x));
    if constexpr (G >= 32) {
        auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
        x = fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
    }
    if constexpr (G == 64) {
        auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
        x = fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
    }
    return x;
}


template <int G>
__device__ __forceinline__ uint32_t group_bcast(uint32_t v, int lane) {
    return static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute((lane & ~(G - 1)) << 2, static_cast<int>(v)));
}

// Next sequence index for the whole group (one atomic by the group leader, broadcast).  Indices
// below `first` (the grid's lane groups) are handed out statically: a group's first sequence is its
// own group number, so a wave starts without an atomic round trip.
// Branch-free on purpose: with `if (leader) v = atomicAdd(...)` the ROCm 7.2 optimiser unswitched
// a loop containing this on `leader` into per-lane copies; the non-leader copy lost the atomic and
// its ds_bpermute read a lane that was not executing (a launch that spun forever on index 0).
// Every lane issues the atomic with increment leader ? 1 : 0; the wave-level atomic optimiser turns
// that into one atomic per wave.
template <int G>
__device__ __forceinline__ uint32_t group_take(uint32_t* counter, bool leader, int lane, uint32_t first) {
    const uint32_t v = atomicAdd(counter, leader ? 1u : 0u);
    return group_bcast<G>(v, lane) + first;
}

}  // namespace

// Per-lane state of one sequence being scored (one "stream"): S match states of the DP row in
// VGPRs, the specials, and the residue cursor.  Separate objects (never an indexed array) so all of
// it stays in registers.
// Rows of residue prefetch: a row of a small profile is short (S=8: ~45 VALU), so the byte load
// for a row is issued RPF rows ahead to cover the L2/HBM latency.
template <int S>
constexpr int residue_prefetch() {
    return S <= 16 ? 6 : (S <= 40 ? 3 : 1);
}

// J and C are kept as PER-LANE partials: J_l = max(J_l' + loop, Elane + tEJ) with Elane the max over
// the lane's own states.  Because max is exact and fl() is monotone, max_l J_l equals the
// reference's J = max(J' + loop, E + tEJ) at every row (induction on the row), so the group-wide
// E is never formed per row; the group max is taken only when B needs J (below) and once at the
// end of the sequence for C.
template <int S, int RPF_ = residue_prefetch<S>()>
struct Stream {
    static constexpr int RPF = RPF_;
    float M[S];
    float J, C, N, B, loop, move;
    float nbr;        // M_{j-1} of the lane's first state; lane 0 of each DPP row is never written
                      // by the shift (invalid source), so it keeps the -inf set once at start
    // pos: residue of the current row; endpos: last residue (prefetch clamp); endp: pos after the
    // last row; ev: pos at which the next event fires (the half-way index fetch, then endp)
    uint32_t pos, endpos, endp, ev, seq;
    uint8_t r[RPF];   // residue codes of the next RPF rows (bytes: a 32-bit slot made the compiler
                      // zero-extend each load where it lands, i.e. wait for it in the same row)
    uint32_t cur;     // BLK: residue blocks, lane b of each 16-lane DPP row = the row of phase b
    uint8_t nxt;      // (cur: this 16-row block, clamped to the poison row; nxt: the next one, raw --
                      // a byte for the reason above, so its load is waited for only where it is used)
    bool active;
    bool junk;        // current "sequence" is an empty/too-long record: discard its row
};

// Per-row working set of one stream.
template <int PF>
struct RowCtx {
    static constexpr int kPF = PF;
    const float4* ep;
    float Bt, nbr, p0, p1, p2, p3;  // (p2, p3 unused: keeping them keeps the register assignment measured in round 1)
    uint8_t rnext;   // residue code RPF rows ahead
    float4 ring[PF];
};

// SA > 0 selects the SPLIT layout (G = 32 or 64, tables too large for LDS): lane gl still owns the S
// consecutive states gl*S+1 .. gl*S+S; its first SA states (the "A block") have all 20 residue rows in
// LDS, its last S - SA states (the "B block") are read from the global table (L2) for every row -- no
// per-row LDS/L2 class branch, so the groups of a wave run the same row body whatever their residues;
// the next row's B halves are requested one row ahead.
// RPFO > 0 overrides the rows of residue prefetch (the zero-copy twins below).
template <int G, int S, int WAVES, int PF, bool BIG, int D, int SA = 0, int RPFO = 0>
__global__ __launch_bounds__(WAVES * 64) void msv_batch_kernel(const KernelArgs a) {
#define MSV_BLOCK blockIdx.x
#define MSV_BLOCKS gridDim.x
#include "msv_kernel_body.inc"
#undef MSV_BLOCK
#undef MSV_BLOCKS
}

// Several profiles' batches in ONE launch (msv_score_grid of a few sequences: each profile's own
// launch would last one sequence's rows, and separate launches serialise on the process's few hardware
// queues).  Workgroups [p * per_profile, (p + 1) * per_profile) score profile p with g.p[p] -- its
// table in this variant's layout, its counter slot, scores and specials -- exactly as msv_batch_kernel
// would with a grid of per_profile workgroups.  The arguments travel in the kernarg segment (copied
// at launch: nothing for the host to keep alive).
template <int G, int S, int WAVES, int PF, bool BIG, int D, int SA = 0, int RPFO = 0>
__global__ __launch_bounds__(WAVES * 64) void msv_grid_kernel(const GridArgs g) {
    const uint32_t profile = blockIdx.x / g.per_profile;
    const uint32_t per_profile = g.per_profile;
    const uint32_t block_in_profile = blockIdx.x - profile * per_profile;
    const KernelArgs a = g.p[profile];
#define MSV_BLOCK block_in_profile
#define MSV_BLOCKS per_profile
#include "msv_kernel_body.inc"
#undef MSV_BLOCK
#undef MSV_BLOCKS
}

// The grid kernel exists for the one-sequence-per-wave (G = 64) variants only: the plans that a few
// sequences take.
template <int G, int S, int WAVES, int PF, bool BIG, int D, int SA = 0>
constexpr const void* grid_fn() {
    if constexpr (G == 64 && D == 1) return reinterpret_cast<const void*>(&msv_grid_kernel<G, S, WAVES, PF, BIG, D, SA>);
    else return nullptr;
}

// Zero-copy twins: the same variant reading its residues two rows ahead -- which for 16/32-lane rows
// means residue BLOCKS (one byte load per lane per 16 rows, a block ahead) -- for launches whose
// residues sit in page-locked host memory.  A row of 41-96 states is long enough that one row of
// prefetch hides an HBM/L2 load, not a PCIe round trip at each 128-B line: cfg3 read in place 2.945 vs
// 2.856 ms with the twin, while from HBM it is 0.3-0.7% slower on 1400/1901.hmm (2% faster on
// 1001.hmm) -- profiles/r02_zero_copy_twins.jsonl.  Split variants already prefetch two rows.
template <int G, int S, int WAVES, int PF, bool BIG, int D, int SA = 0>
constexpr const void* zc_fn() {
    if constexpr ((G == 16 || G == 32) && D == 1 && !BIG && SA == 0 && S > 40)
        return reinterpret_cast<const void*>(&msv_batch_kernel<G, S, WAVES, PF, BIG, D, SA, 2>);
    else return nullptr;
}

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
// part: 16 words of LDS).  hist is read with device-scope loads: the other blocks' counts
// arrived by atomics at L2.
__device__ __forceinline__ void scan_bins(uint32_t* __restrict__ hist, uint32_t* __restrict__ cursor, uint32_t nbins,
                                          uint32_t* part) {
    const uint32_t t = threadIdx.x;
    uint32_t v[4], sum = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t i = 4 * t + q;
        v[q] = i < nbins ? __hip_atomic_load(&hist[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        if (i < nbins) hist[i] = 0u;
        sum += v[q];
    }
    uint32_t run = block_exclusive_sum(sum, part);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t i = 4 * t + q;
        if (i < nbins) cursor[i] = run;
        run += v[q];
    }
}

// scratch = [hist | cursor | ticket]; the last block to add its counts runs the scan, and no block
// waits for another.  The hand-off needs no fences: the counts are agent-scope atomics (performed past
// the XCD's L2), every wave drains them (vmcnt) before the block's ticket add, and the block whose add
// returns the last ticket reads them with sc1 loads after a barrier (MI355X_MICROARCH.md,
// inter-workgroup visibility, first row of the sc1 hand-offs).  A __threadfence() in every block
// (L2 write-back + invalidate) made this launch 57 us instead of 5.
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
    scan_bins(hist, scratch + nbins, nbins, lh);
    if (threadIdx.x == 0) scratch[2 * nbins] = 0u;
}

__global__ __launch_bounds__(kOrderThreads) void order_place_kernel(const uint64_t* __restrict__ offsets, uint64_t n,
                                                                    uint64_t chunk, uint32_t* __restrict__ cursor,
                                                                    uint32_t nbins, uint32_t* __restrict__ order) {
    extern __shared__ uint32_t lh[];  // [0, nbins): block counts, then block cursors
    for (uint32_t i = threadIdx.x; i < nbins; i += blockDim.x) lh[i] = 0;
    __syncthreads();
    const uint64_t lo = blockIdx.x * chunk, hi = min(n, lo + chunk);
    for (uint64_t s = lo + threadIdx.x; s < hi; s += blockDim.x) atomicAdd(&lh[length_bin(offsets, s, nbins)], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nbins; i += blockDim.x)
        if (lh[i]) lh[i] = atomicAdd(&cursor[i], lh[i]);  // reserve this block's range of bin i
    __syncthreads();
    for (uint64_t s = lo + threadIdx.x; s < hi; s += blockDim.x) {
        const uint32_t slot = atomicAdd(&lh[length_bin(offsets, s, nbins)], 1u);
        order[slot] = static_cast<uint32_t>(s);
    }
}

// ------------------------------------------------------------------------------------------------
// MSV filter P-values (msv.h): one thread per sequence, HBM-bound elementwise
// (12 B read + 8 B written per sequence).  Same float/double steps as msv_stats.cpp's host path.
// ------------------------------------------------------------------------------------------------
__device__ __host__ inline double msv_pvalue_of(float score, uint64_t L, float mu, float lambda) {
    if (L == 0) return 1.0;  // empty sequence: score -inf, and L log(p1) would be 0 * -inf
    const float p1 = static_cast<float>(L) / static_cast<float>(L + 1);
    const float nullsc = static_cast<float>(static_cast<double>(L) * log(static_cast<double>(p1)) +
                                            log(1.0 - static_cast<double>(p1)));
    const float bits = (score - nullsc) / 0.69314718055994529f;
    const double y = static_cast<double>(lambda) * (static_cast<double>(bits) - static_cast<double>(mu));
    const double ey = -exp(-y);
    return fabs(ey) < 5e-9 ? -ey : 1.0 - exp(ey);
}

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
// Variant table: every compiled (G, S, WAVES) instantiation.  The host picks the one whose G*S
// covers LENG with the least estimated cost (the analog of the reference's should_specialize,
// which bakes sizes into the OpenCL program with -D defines, MSV_HMM.cpp:322-337).
// ------------------------------------------------------------------------------------------------
#define MSV_VARIANT(G_, S_, W_, P_, D_)                                                                   \
    Variant{G_, S_, W_, P_, D_, lds_rows_for(G_, S_), lds_rows_for(G_, S_) < kTableRows,                  \
            reinterpret_cast<const void*>(                                                                 \
                &msv_batch_kernel<G_, S_, W_, P_, (lds_rows_for(G_, S_) < kTableRows), D_>),               \
            "msv_g" #G_ "_s" #S_ "_w" #W_ "_p" #P_ "_d" #D_, 0,                                              \
            grid_fn<G_, S_, W_, P_, (lds_rows_for(G_, S_) < kTableRows), D_>(),                            \
            zc_fn<G_, S_, W_, P_, (lds_rows_for(G_, S_) < kTableRows), D_>()}

// Split layout (G = 32 or 64): SA states per lane from LDS (20 rows), S - SA from L2.
#define MSV_SPLIT_VARIANT(G_, S_, SA_, W_, P_)                                                            \
    Variant{G_, S_, W_, P_, 1, kAminoAcids, false,                                                        \
            reinterpret_cast<const void*>(&msv_batch_kernel<G_, S_, W_, P_, false, 1, SA_>),               \
            "msv_g" #G_ "_s" #S_ "_a" #SA_ "_w" #W_ "_p" #P_ "_d1", SA_, grid_fn<G_, S_, W_, P_, false, 1, SA_>()}

static const Variant kVariants[] = {
#include "msv_variants.inc"
};

const Variant* variants(int* count) {
    *count = static_cast<int>(sizeof(kVariants) / sizeof(kVariants[0]));
    return kVariants;
}

hipError_t launch_variant(const Variant& v, dim3 grid, const KernelArgs& args, hipStream_t stream, hipEvent_t start,
                          hipEvent_t stop, bool host_residues) {
    void* params[] = {const_cast<KernelArgs*>(&args)};
    const void* fn = host_residues && v.zc_fn ? v.zc_fn : v.fn;
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
