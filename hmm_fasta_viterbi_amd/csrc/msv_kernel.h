// msv_kernel.h -- device-side interface shared by msv_kernel.hip and the C-ABI layer.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace msvk {

constexpr int kAminoAcids = 20;
constexpr int kPoisonRow = 20;   // codes >= 20 are clamped here; the row is +inf -> score +inf -> error
constexpr int kTableRows = 21;   // 20 residues + poison row
// RPFO value (msv_batch_kernel's last template parameter) that selects the wide-block zero-copy twin
// of a residue-block variant (msv_kernel_impl.h zc_fn)
constexpr int kWideBlocks = 64;
constexpr int kLdsLimit = 163840;

// Words per wave of the diagnostic stamps buffer (KernelArgs::stamps): realtime start/end, hwid|rows,
// xcc|block (4 words in the production kernels), and in the CLOCK twins shader-clock (s_memtime) start/end.
constexpr int kStampWords = 6;
// RPFO value that selects a variant's CLOCK twin: the same kernel whose stamps also record shader-clock
// ticks (bench.py's clock_GHz).  A separate instantiation, so the production kernels' ISA is untouched.
constexpr int kClockTwin = -1;

constexpr uint32_t kErrBadResidue = 1u;
constexpr uint32_t kErrTooLong = 2u;
constexpr uint32_t kErrBadOrder = 4u;  // a dequeue-order entry >= n (caller's order, or a poisoned sort)
constexpr uint32_t kErrTeamHang = 8u;  // a Viterbi team's LDS exchange never completed (vit_team.hip; a bug)

// Residue rows of the [row][chunk][lane] float4 table that fit the 160 KiB LDS of one CU.
constexpr int lds_rows_for(int G, int S) {
    return (kLdsLimit / (G * S * 4)) >= kTableRows ? kTableRows : (kLdsLimit / (G * S * 4));
}

// MSV filter P-value of one score (HMMER3's MSV-stage formula, msv.h msv_pvalues): used by the P-value
// kernel, the host path and the Viterbi stage's survivor selection (vit_kernel.hip).
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

struct KernelArgs {
    const float4* etab;        // [21][S/4][G] float4, global copy of the kernel-layout table
    const uint8_t* residues;   // CSR residue codes
    const uint64_t* offsets;   // n + 1
    const uint32_t* order;     // optional dequeue permutation (n) or nullptr
    const float2* lentab;      // [lentab_n] {tr_loop, tr_move} indexed by sequence length
    float* scores;             // n
    uint32_t* counter;         // dequeue head, zeroed before each launch
    uint32_t* errors;          // sticky error bits
    uint64_t n;
    uint32_t lentab_n;
    float tr_B_Mk, tr_E_C, tr_E_J;
    uint64_t* stamps;          // diagnostic per-wave timeline (nullptr in production)
};

// One launch over several profiles (msv_grid_kernel): profile k runs p[k] on workgroups
// [k * per_profile, (k + 1) * per_profile).  Passed by value (kernarg segment, < 4 KiB).
constexpr uint32_t kGridMaxProfiles = 32;
struct GridArgs {
    uint32_t profiles;
    uint32_t per_profile;
    KernelArgs p[kGridMaxProfiles];
};
static_assert(sizeof(GridArgs) <= 4096, "kernel arguments are limited to 4 KiB");

struct Variant {
    int G, S, waves, pf, streams;  // pf = emission ring depth; streams = sequences per lane group
    int lds_rows;
    bool big;
    const void* fn;
    const char* name;
    int sa = 0;  // split layout: states per lane staged in LDS (0 = whole table layout)
    const void* grid_fn = nullptr;  // msv_grid_kernel instantiation (G = 64 variants), else nullptr
    const void* zc_fn = nullptr;    // zero-copy twin (residues two rows ahead), else nullptr
    const void* clock_fn = nullptr; // CLOCK twin (stamps record shader-clock ticks; bench configs' plans only)
};

const Variant* variants(int* count);

// The cooperative plan (msv_coop.hip): one sequence per workgroup of `waves` waves, each wave holding
// 64 lanes x S states of the row, the first `halo` of them a redundant copy of the previous wave's last
// states.  Wave w's lane l, state q covers global state w * (64 S - halo) - halo + l S + q + 1; the table
// is [21 rows][waves][S / 2][64 lanes] float2, staged whole in LDS.
// sa < S (split): the lane's first sa states in that LDS table ([21][waves][sa / 2][64] float2), its last
// S - sa from a global table [21][waves][64][S - sa] floats that follows it.
struct CoopVariant {
    int waves, S, halo;
    const void* fn;
    const char* name;
    int sa;
    const void* grid_fn;  // msv_coop_grid_kernel: several profiles' batches in one launch (GridArgs)
    int states() const { return waves * (64 * S - halo); }
};
const CoopVariant* coop_variants(int* count);
// start/stop (optional): events updated with the kernel's own start and end (hipExtLaunchKernel), so a
// timed launch costs no extra marker packets on the stream.
// host_residues: args.residues is the device alias of page-locked host memory (the zero-copy twin
// runs when the variant has one).
// clock: run the variant's CLOCK twin (args.stamps set, kStampWords per wave); the caller checks clock_fn.
hipError_t launch_variant(const Variant& v, dim3 grid, const KernelArgs& args, hipStream_t stream,
                          hipEvent_t start = nullptr, hipEvent_t stop = nullptr, bool host_residues = false,
                          bool clock = false);
// Several profiles in one launch (v.grid_fn must be set).
hipError_t launch_grid_variant(const Variant& v, const GridArgs& args, hipStream_t stream);
hipError_t launch_pvalues(const float* scores, const uint64_t* offsets, uint64_t n, float mu, float lambda,
                          double* pvalues, hipStream_t stream);

// scratch_hist: kOrderScratchWords(nbins) words [histogram | cursors | ticket | bad]; histogram and ticket must
// be zero on entry and are zero again when the sort completes (zero them once when fresh, or after a
// failed launch).  1024 <= nbins <= 4096 (the scan runs 1024 threads over 4 bins each).
constexpr uint32_t kOrderScratchWords(uint32_t nbins) { return 2 * nbins + 64; }
hipError_t launch_order(const uint64_t* offsets, uint64_t n, uint32_t* scratch_hist, uint32_t nbins, uint32_t* order,
                        hipStream_t stream);

}  // namespace msvk
