// fasta_device.hip -- FASTA ingest on the GPU: raw FASTA bytes in HBM -> the CSR
// residue stream the MSV kernel consumes, with the record semantics of the reference reader
// (FASTA_protein_sequences.cpp:9-44, restated by host_parsers.cpp:parse_fasta_chunk):
//   * a line starting with '>' opens a record (header = rest of the line, '\r' kept);
//   * every other line is appended to the open record; a record holding any byte outside
//     {20 amino acids, '#'} is dropped ('#' becomes code 255, rejected later by the scorer);
//   * empty records are kept; empty lines anywhere are ignored; a non-empty line before the first
//     header is MSV_ERR_PARSE.
//
// Byte work, HBM-bound, no MFMA.  Every byte's role depends on the line it sits in (header or
// not) and on how many headers / residue bytes precede it, so the parse is a set of scans over
// 8 KiB tiles (one 256-thread block, 32 bytes per thread read as two uint4):
//   1. fa_tile_summary  per tile: header starts, position of its last line start, residue bytes
//                       decidable locally, bytes of the leading partial line (whose header-ness
//                       comes from an earlier tile);
//   2. scan (sum, max)  exclusive over tiles: header starts before the tile, last line start before
//                       it -> fa_tile_carry: the open line's header-ness and the tile's residue
//                       count -> scan (sum): residue bytes before the tile;
//   3. fa_tile_emit     per tile again, now with exact carries: every residue byte is translated and
//                       written at its rank, records get their residue start / header span, a bad
//                       byte marks its record rejected;
//   4. fa_rec_values -> scan (sum, sum) -> fa_rec_write: kept-record offsets (uint64 CSR), header
//                       spans, compaction sources, counts;
//   5. fa_compact       only when a record was rejected: kept records' residues moved to the final
//                       stream, one wave per record.
// Every scan is the 3-launch hierarchical kind (block reduce -> one-block scan of the block
// partials -> block down-sweep), 4096 elements per 256-thread block.
// Positions are uint32 (n < 2^32 - 2^16 bytes per call; the scorer's residue stream is uint32 too).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "msv.h"

namespace fadev {

constexpr int kThreads = 256;
constexpr int kPerThread = 16;                     // scan elements per thread
constexpr uint32_t kTile = kThreads * kPerThread;  // scan elements per block (4096)
constexpr int kBytesPerThread = 32;                // text bytes per thread (two uint4 loads)
constexpr uint32_t kTileBytes = kThreads * kBytesPerThread;  // 8 KiB of text per block
constexpr int kScanThreads = 1024;
constexpr uint32_t kUnset = 0xFFFFFFFFu;
constexpr uint8_t kBad = 254;
constexpr uint64_t kMaxText = 0xFFFF0000ull;  // uint32 positions, tile indices stay in range

struct ResidueLut {
    uint8_t v[256];
};
constexpr ResidueLut make_lut() {
    ResidueLut l{};
    for (int i = 0; i < 256; ++i) l.v[i] = kBad;
    const char* letters = "ACDEFGHIKLMNPQRSTVWY";  // MSV_HMM.cpp:29-31
    for (int i = 0; i < 20; ++i) l.v[static_cast<unsigned char>(letters[i])] = static_cast<uint8_t>(i);
    l.v[static_cast<unsigned char>('#')] = 255;
    return l;
}
// In global memory, not __constant__: a per-lane (divergent) index into constant memory is lowered
// to a scalar-load waterfall loop; kernels copy this into LDS and index it there.
__device__ const ResidueLut kLut = make_lut();

struct TileCarry {
    uint32_t hdr_in;  // header-ness of the line open at the tile's first byte
    uint32_t h_excl;  // header starts before the tile
    uint32_t r_excl;  // residue bytes before the tile
    uint32_t pad;
};

struct Totals {
    uint32_t headers;   // records seen (header starts)
    uint32_t residues;  // residue bytes incl. rejected records'
    uint32_t kept;      // records kept
    uint32_t kept_res;  // residues of kept records
    uint32_t error;     // bit0: residue bytes before the first header
    uint32_t max_len;   // longest kept record
    uint32_t pad[2];
};

__device__ __forceinline__ void load32(const uint8_t* __restrict__ T, uint32_t n, uint32_t i0,
                                       uint8_t (&b)[kBytesPerThread]) {
    if (i0 + kBytesPerThread <= n && (reinterpret_cast<uintptr_t>(T + i0) & 15) == 0) {
#pragma unroll
        for (int h = 0; h < kBytesPerThread / 16; ++h) {
            const uint4 v = *reinterpret_cast<const uint4*>(T + i0 + 16 * h);
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int k = 0; k < 16; ++k) b[16 * h + k] = static_cast<uint8_t>(w[k >> 2] >> (8 * (k & 3)));
        }
    } else {
#pragma unroll
        for (int k = 0; k < kBytesPerThread; ++k) b[k] = i0 + k < n ? T[i0 + k] : static_cast<uint8_t>('\n');
    }
}

// A thread's 32 bytes as bit masks (bit k = byte i0 + k): branch-free per-byte work, no SGPR-mask
// explosion from 32 unrolled data-dependent branches.
struct ByteMasks {
    uint32_t valid, nl, ls, hs;  // in range, '\n', line start, header start ('>' at a line start)
};

__device__ __forceinline__ ByteMasks byte_masks(const uint8_t (&b)[kBytesPerThread], uint8_t prev, uint32_t i0,
                                                uint32_t n) {
    ByteMasks m{0, 0, 0, 0};
    m.valid = i0 >= n ? 0u : (n - i0 >= 32u ? 0xFFFFFFFFu : ((1u << (n - i0)) - 1u));
    uint32_t gt = 0;
#pragma unroll
    for (int k = 0; k < kBytesPerThread; ++k) {
        m.nl |= static_cast<uint32_t>(b[k] == '\n') << k;
        gt |= static_cast<uint32_t>(b[k] == '>') << k;
    }
    m.nl &= m.valid;
    m.ls = ((m.nl << 1) | static_cast<uint32_t>(prev == '\n')) & m.valid;
    m.hs = m.ls & gt;
    return m;
}

// Bytes whose line is a header line, given whether the line open at the thread's first byte is one.
__device__ __forceinline__ uint32_t header_line_mask(const ByteMasks& m, bool hdr_in) {
    uint32_t st = hdr_in ? 1u : 0u, out = 0;
#pragma unroll
    for (int k = 0; k < kBytesPerThread; ++k) {
        const uint32_t ls = (m.ls >> k) & 1u;
        st = ls ? ((m.hs >> k) & 1u) : st;
        out |= st << k;
    }
    return out;
}

__device__ __forceinline__ uint32_t below(int k) { return k >= 32 ? 0xFFFFFFFFu : ((1u << k) - 1u); }

struct ThreadFacts {
    uint32_t hs, pre, res_after, last_ls;  // last_ls: tile-local position of the last line start
    bool has_ls, last_hdr;
};

__device__ __forceinline__ ThreadFacts thread_facts(const ByteMasks& m, uint32_t i0, uint32_t t0) {
    ThreadFacts f{};
    const uint32_t nonnl = m.valid & ~m.nl;
    f.has_ls = m.ls != 0;
    const uint32_t prefix = f.has_ls ? below(__builtin_ctz(m.ls)) : 0xFFFFFFFFu;  // bytes before the first LS
    f.pre = __builtin_popcount(nonnl & prefix);
    f.res_after = __builtin_popcount(nonnl & ~prefix & ~header_line_mask(m, false));
    f.hs = __builtin_popcount(m.hs);
    if (f.has_ls) {
        const int k = 31 - __builtin_clz(m.ls);
        f.last_ls = i0 + k - t0;
        f.last_hdr = (m.hs >> k) & 1u;
    }
    return f;
}

// ---- wave-level DPP scans (64 lanes) and their block-level composition ---------------------------
template <int CTRL, int ROW_MASK, bool BOUND0>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x) {
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), CTRL, ROW_MASK, 0xF, BOUND0));
}

// Inclusive scan over the wave: row_shr 1/2/4/8 inside each 16-lane row (invalid lanes read 0),
// then row_bcast:15 / row_bcast:31 carry the row totals up.  OP 0 = add, 1 = max (identity 0).
template <int OP>
__device__ __forceinline__ uint32_t wave_inclusive(uint32_t x) {
    auto f = [](uint32_t a, uint32_t b) { return OP ? max(a, b) : a + b; };
    x = f(x, dpp_u32<0x111, 0xF, true>(x));
    x = f(x, dpp_u32<0x112, 0xF, true>(x));
    x = f(x, dpp_u32<0x114, 0xF, true>(x));
    x = f(x, dpp_u32<0x118, 0xF, true>(x));
    x = f(x, dpp_u32<0x142, 0xA, false>(x));
    x = f(x, dpp_u32<0x143, 0xC, false>(x));
    return x;
}

// Block-wide exclusive scan (add or max) of one uint32 per thread; `total` = block aggregate.
// SLOT gives each scan of a kernel its own LDS exchange array (no barrier needed between them).
template <int OP, int SLOT>
__device__ __forceinline__ uint32_t block_exclusive_u32(uint32_t x, uint32_t& total) {
    __shared__ uint32_t wtot[kThreads / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t inc = wave_inclusive<OP>(x);
    // exclusive inside the wave: the previous lane's inclusive value (wave_shr:1, lane 0 reads 0)
    const uint32_t exw =
        static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(inc), 0x138, 0xF, 0xF, true));
    if (lane == 63) wtot[wave] = inc;
    __syncthreads();
    uint32_t base = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) {
        const uint32_t v = wtot[w];
        if (w < wave) base = OP ? max(base, v) : base + v;
        all = OP ? max(all, v) : all + v;
    }
    total = all;
    return OP ? max(base, exw) : base + exw;
}

__global__ __launch_bounds__(kThreads) void fa_tile_summary(const uint8_t* __restrict__ T, uint32_t n,
                                                            uint2* __restrict__ hs_ls, uint2* __restrict__ pre_res) {
    const uint32_t t0 = blockIdx.x * kTileBytes;
    const uint32_t i0 = t0 + threadIdx.x * kBytesPerThread;
    uint8_t b[kBytesPerThread];
    load32(T, n, i0, b);
    const uint8_t prev = i0 == 0 ? static_cast<uint8_t>('\n') : (i0 - 1 < n ? T[i0 - 1] : static_cast<uint8_t>('\n'));
    const ByteMasks bm = byte_masks(b, prev, i0, n);
    const ThreadFacts f = thread_facts(bm, i0, t0);
    // last line start before this thread: (tile-local position + 1) << 1 | header bit, 0 = none
    uint32_t ls_tot;
    const uint32_t ls = block_exclusive_u32<1, 0>(f.has_ls ? (((f.last_ls + 1) << 1) | (f.last_hdr ? 1u : 0u)) : 0u,
                                                  ls_tot);
    const bool cv = ls != 0, ch = ls & 1u;
    // bytes before this thread's first line start: tile prefix if no earlier thread had a line
    // start, otherwise residue iff that line is not a header
    const uint32_t pre_tile = cv ? 0u : f.pre;
    const uint32_t res = f.res_after + ((cv && !ch) ? f.pre : 0u);
    uint32_t s_hr, s_pre;
    (void)block_exclusive_u32<0, 1>(f.hs | (res << 16), s_hr);  // both < 2^16 per tile
    (void)block_exclusive_u32<0, 2>(pre_tile, s_pre);
    if (threadIdx.x == 0) {
        const uint32_t last_ls = ls_tot ? t0 + (ls_tot >> 1) : 0u;  // 1 + absolute position, 0 = none
        hs_ls[blockIdx.x] = make_uint2(s_hr & 0xFFFFu, last_ls);
        pre_res[blockIdx.x] = make_uint2(s_pre, s_hr >> 16);
    }
}

// Per tile, once the line-start and header-start scans are known: the header-ness of the line open
// at the tile's first byte (the line of the last line start before the tile) and the tile's
// residue count.
__global__ __launch_bounds__(kThreads) void fa_tile_carry(const uint8_t* __restrict__ T, uint32_t nt,
                                                          const uint2* __restrict__ hs_ls_excl,
                                                          const uint2* __restrict__ pre_res, uint2* __restrict__ res,
                                                          TileCarry* __restrict__ carry) {
    const uint32_t t = blockIdx.x * kThreads + threadIdx.x;
    if (t >= nt) return;
    const uint2 ex = hs_ls_excl[t];
    const uint32_t hdr_in = ex.y ? (T[ex.y - 1] == '>') : 0u;
    const uint2 pr = pre_res[t];
    res[t] = make_uint2(pr.y + (hdr_in ? 0u : pr.x), 0u);
    carry[t].hdr_in = hdr_in;
    carry[t].h_excl = ex.x;
}

// r_excl from the residue scan.
__global__ __launch_bounds__(kThreads) void fa_tile_rexcl(uint32_t nt, const uint2* __restrict__ res_excl,
                                                          TileCarry* __restrict__ carry) {
    const uint32_t t = blockIdx.x * kThreads + threadIdx.x;
    if (t < nt) carry[t].r_excl = res_excl[t].x;
}

__global__ __launch_bounds__(kThreads) void fa_tile_emit(const uint8_t* __restrict__ T, uint32_t n,
                                                         const TileCarry* __restrict__ carry,
                                                         uint8_t* __restrict__ codes, uint32_t* __restrict__ rec_start,
                                                         uint32_t* __restrict__ hdr_start, uint32_t* __restrict__ hdr_end,
                                                         uint8_t* __restrict__ bad, Totals* __restrict__ tot) {
    __shared__ uint8_t stage[kTileBytes];  // this tile's residue codes, written out coalesced
    __shared__ uint8_t lut[256];
    lut[threadIdx.x] = kLut.v[threadIdx.x];  // kThreads == 256; the scans below barrier before use
    const uint32_t t0 = blockIdx.x * kTileBytes;
    const uint32_t i0 = t0 + threadIdx.x * kBytesPerThread;
    uint8_t b[kBytesPerThread];
    load32(T, n, i0, b);
    const uint8_t prev = i0 == 0 ? static_cast<uint8_t>('\n') : (i0 - 1 < n ? T[i0 - 1] : static_cast<uint8_t>('\n'));
    const ByteMasks bm = byte_masks(b, prev, i0, n);
    const ThreadFacts f = thread_facts(bm, i0, t0);
    uint32_t ls_tot;
    const uint32_t ls = block_exclusive_u32<1, 0>(f.has_ls ? (((f.last_ls + 1) << 1) | (f.last_hdr ? 1u : 0u)) : 0u,
                                                  ls_tot);
    const TileCarry tc = carry[blockIdx.x];
    const bool hdr_in = ls ? (ls & 1u) != 0 : (tc.hdr_in != 0);  // header-ness of the line open at i0
    const uint32_t hline = header_line_mask(bm, hdr_in);
    const uint32_t resm = bm.valid & ~bm.nl & ~hline;  // residue bytes
    const uint32_t res = __builtin_popcount(resm);
    uint32_t s_hr;
    const uint32_t ex = block_exclusive_u32<0, 1>(f.hs | (res << 16), s_hr);
    const uint32_t rec0 = tc.h_excl + (ex & 0xFFFFu);  // header starts before i0
    const uint32_t local0 = ex >> 16;                   // this tile's residue bytes before i0
    // residues -> LDS stage at their tile-local rank; rejected-byte mask for the records below
    uint32_t badm = 0;
#pragma unroll
    for (int k = 0; k < kBytesPerThread; ++k) {
        const uint8_t code = lut[b[k]];
        badm |= static_cast<uint32_t>(code == kBad) << k;
        if ((resm >> k) & 1u) stage[local0 + __builtin_popcount(resm & below(k))] = code;
    }
    badm &= resm;
    // records opened here (rare): residue start and header start
    for (uint32_t m = bm.hs; m; m &= m - 1) {
        const int k = __builtin_ctz(m);
        const uint32_t r = rec0 + __builtin_popcount(bm.hs & below(k));
        rec_start[r] = tc.r_excl + local0 + __builtin_popcount(resm & below(k));
        hdr_start[r] = i0 + k + 1;
    }
    // header lines ended here: the newline of a header line
    for (uint32_t m = bm.nl & hline; m; m &= m - 1) {
        const int k = __builtin_ctz(m);
        hdr_end[rec0 + __builtin_popcount(bm.hs & below(k + 1)) - 1] = i0 + k;
    }
    // rejected records (a byte outside the alphabet) and residues before the first header
    bool pre_header_bytes = false;
    for (uint32_t m = badm; m; m &= m - 1) {
        const int k = __builtin_ctz(m);
        const uint32_t r = rec0 + __builtin_popcount(bm.hs & below(k + 1));
        if (r) bad[r - 1] = 1;
    }
    if (rec0 == 0) {
        const uint32_t before_first_hs = bm.hs ? below(__builtin_ctz(bm.hs)) : 0xFFFFFFFFu;
        pre_header_bytes = (resm & before_first_hs) != 0;
    }
    if (pre_header_bytes) atomicOr(&tot->error, 1u);
    __syncthreads();
    // coalesced copy-out: bytes up to a 4-byte boundary of the output, then words, then the tail
    const uint32_t count = s_hr >> 16;
    uint8_t* __restrict__ out = codes + tc.r_excl;
    const uint32_t head = min(count, (4u - (tc.r_excl & 3u)) & 3u);
    if (threadIdx.x < head) out[threadIdx.x] = stage[threadIdx.x];
    const uint32_t words = (count - head) >> 2;
    uint32_t* __restrict__ outw = reinterpret_cast<uint32_t*>(out + head);
    for (uint32_t j = threadIdx.x; j < words; j += kThreads) {
        const uint32_t o = head + 4 * j;
        outw[j] = static_cast<uint32_t>(stage[o]) | (static_cast<uint32_t>(stage[o + 1]) << 8) |
                  (static_cast<uint32_t>(stage[o + 2]) << 16) | (static_cast<uint32_t>(stage[o + 3]) << 24);
    }
    const uint32_t tail = head + 4 * words;
    if (tail + threadIdx.x < count) out[tail + threadIdx.x] = stage[tail + threadIdx.x];
}

// ---- hierarchical exclusive scan of uint2 elements; OPX / OPY: 0 = sum, 1 = max (identity 0) ----
template <int OPX, int OPY>
__device__ __forceinline__ uint2 comb(uint2 a, uint2 b) {
    return make_uint2(OPX ? max(a.x, b.x) : a.x + b.x, OPY ? max(a.y, b.y) : a.y + b.y);
}

template <int OPX, int OPY>
__device__ __forceinline__ uint2 block_exclusive(uint2 v, uint2& total) {
    __shared__ uint2 s[kThreads];
    const int t = threadIdx.x;
    s[t] = v;
    __syncthreads();
    uint2 acc = v;
    for (int d = 1; d < kThreads; d <<= 1) {
        const uint2 o = t >= d ? s[t - d] : make_uint2(0, 0);
        __syncthreads();
        acc = comb<OPX, OPY>(o, acc);
        s[t] = acc;
        __syncthreads();
    }
    total = s[kThreads - 1];
    const uint2 ex = t > 0 ? s[t - 1] : make_uint2(0, 0);
    __syncthreads();
    return ex;
}

template <int OPX, int OPY>
__global__ __launch_bounds__(kThreads) void scan_reduce(const uint2* __restrict__ in, uint32_t n,
                                                        uint2* __restrict__ part) {
    const uint32_t base = blockIdx.x * kTile + threadIdx.x * kPerThread;
    uint2 acc = make_uint2(0, 0);
#pragma unroll
    for (int k = 0; k < kPerThread; ++k)
        if (base + k < n) acc = comb<OPX, OPY>(acc, in[base + k]);
    uint2 total;
    (void)block_exclusive<OPX, OPY>(acc, total);
    if (threadIdx.x == 0) part[blockIdx.x] = total;
}

template <int OPX, int OPY>
__global__ __launch_bounds__(kScanThreads) void scan_partials(uint2* __restrict__ part, uint32_t np) {
    __shared__ uint2 s[kScanThreads];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (np + kScanThreads - 1) / kScanThreads;
    const uint32_t a = min(np, t * per), b = min(np, a + per);
    uint2 acc = make_uint2(0, 0);
    for (uint32_t k = a; k < b; ++k) acc = comb<OPX, OPY>(acc, part[k]);
    s[t] = acc;
    __syncthreads();
    uint2 v = acc;
    for (uint32_t d = 1; d < kScanThreads; d <<= 1) {
        const uint2 o = t >= d ? s[t - d] : make_uint2(0, 0);
        __syncthreads();
        v = comb<OPX, OPY>(o, v);
        s[t] = v;
        __syncthreads();
    }
    uint2 run = t > 0 ? s[t - 1] : make_uint2(0, 0);
    for (uint32_t k = a; k < b; ++k) {
        const uint2 x = part[k];
        part[k] = run;
        run = comb<OPX, OPY>(run, x);
    }
}

template <int OPX, int OPY>
__global__ __launch_bounds__(kThreads) void scan_down(const uint2* __restrict__ in, uint32_t n,
                                                      const uint2* __restrict__ part, uint2* __restrict__ out) {
    const uint32_t base = blockIdx.x * kTile + threadIdx.x * kPerThread;
    uint2 v[kPerThread];
    uint2 acc = make_uint2(0, 0);
#pragma unroll
    for (int k = 0; k < kPerThread; ++k) {
        v[k] = base + k < n ? in[base + k] : make_uint2(0, 0);
        acc = comb<OPX, OPY>(acc, v[k]);
    }
    uint2 total;
    uint2 run = comb<OPX, OPY>(part[blockIdx.x], block_exclusive<OPX, OPY>(acc, total));
#pragma unroll
    for (int k = 0; k < kPerThread; ++k) {
        if (base + k < n) out[base + k] = run;
        run = comb<OPX, OPY>(run, v[k]);
    }
}

// Per record: (kept, kept residues) for the offsets scan.
__global__ __launch_bounds__(kThreads) void fa_rec_values(uint32_t nrec, const uint32_t* __restrict__ rec_start,
                                                          const uint8_t* __restrict__ bad,
                                                          const Totals* __restrict__ tot, uint2* __restrict__ v) {
    const uint32_t r = blockIdx.x * kThreads + threadIdx.x;
    if (r >= nrec) return;
    const uint32_t end = r + 1 < nrec ? rec_start[r + 1] : tot->residues;
    const bool keep = !bad[r];
    v[r] = make_uint2(keep ? 1u : 0u, keep ? end - rec_start[r] : 0u);
}

// Per kept record: CSR offset, header span, compaction source; the last record writes the totals.
__global__ __launch_bounds__(kThreads) void fa_rec_write(uint32_t nrec, uint32_t n, const uint2* __restrict__ v,
                                                         const uint2* __restrict__ ex,
                                                         const uint32_t* __restrict__ rec_start,
                                                         const uint32_t* __restrict__ hdr_start,
                                                         const uint32_t* __restrict__ hdr_end,
                                                         uint64_t* __restrict__ offsets, uint64_t* __restrict__ spans,
                                                         uint32_t* __restrict__ src, Totals* __restrict__ tot) {
    const uint32_t r = blockIdx.x * kThreads + threadIdx.x;
    if (r >= nrec) return;
    const uint2 e = ex[r], x = v[r];
    if (x.x) {
        offsets[e.x] = e.y;
        const uint32_t hs = hdr_start[r];
        const uint32_t he = hdr_end[r] == kUnset ? n : hdr_end[r];  // header line ended by EOF
        spans[2ull * e.x] = hs;
        spans[2ull * e.x + 1] = he - hs;
        src[e.x] = rec_start[r];
    }
    if (r == nrec - 1) {
        offsets[e.x + x.x] = e.y + x.y;
        tot->kept = e.x + x.x;
        tot->kept_res = e.y + x.y;
    }
}

// Longest kept record from the per-block maxima of scan_reduce<1, 1> over the record values.
__global__ __launch_bounds__(kScanThreads) void fa_max_partials(const uint2* __restrict__ part, uint32_t np,
                                                                Totals* __restrict__ tot) {
    __shared__ uint32_t s[kScanThreads];
    uint32_t m = 0;
    for (uint32_t k = threadIdx.x; k < np; k += kScanThreads) m = max(m, part[k].y);
    s[threadIdx.x] = m;
    __syncthreads();
    for (uint32_t d = kScanThreads / 2; d > 0; d >>= 1) {
        if (threadIdx.x < d) s[threadIdx.x] = max(s[threadIdx.x], s[threadIdx.x + d]);
        __syncthreads();
    }
    if (threadIdx.x == 0) tot->max_len = s[0];
}

// Totals of the tile pass from the last tile's values.
__global__ void fa_tile_totals(uint32_t nt, const uint2* __restrict__ hs_ls, const uint2* __restrict__ hs_ls_excl,
                               const uint2* __restrict__ res, const uint2* __restrict__ res_excl,
                               Totals* __restrict__ tot) {
    tot->headers = hs_ls_excl[nt - 1].x + hs_ls[nt - 1].x;
    tot->residues = res_excl[nt - 1].x + res[nt - 1].x;
}

// Kept records' residues to their final place (only when a record was rejected): one wave per record.
__global__ __launch_bounds__(kThreads) void fa_compact(const uint8_t* __restrict__ from, uint32_t nkept,
                                                       const uint64_t* __restrict__ offsets,
                                                       const uint32_t* __restrict__ src, uint8_t* __restrict__ to) {
    const uint32_t wave = (blockIdx.x * kThreads + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t waves = (gridDim.x * kThreads) >> 6;
    for (uint32_t k = wave; k < nkept; k += waves) {
        const uint64_t o = offsets[k], L = offsets[k + 1] - o;
        const uint32_t s0 = src[k];
        for (uint64_t j = lane; j < L; j += 64) to[o + j] = from[s0 + j];
    }
}

}  // namespace fadev

// ------------------------------------------------------------------------------------------------
// Host orchestration and C-ABI
// ------------------------------------------------------------------------------------------------
struct msv_fasta_device {
    int device = 0;
    uint64_t count = 0, rejected = 0, residues = 0, max_length = 0;
    uint8_t* d_codes = nullptr;   // final residue stream (either d_stage or d_final)
    uint8_t* d_stage = nullptr;   // residues at their rank (incl. rejected records)
    uint8_t* d_final = nullptr;   // compacted stream (only when a record was rejected)
    uint64_t* d_offsets = nullptr;
    uint64_t* d_spans = nullptr;
    uint8_t* d_text = nullptr;    // owned copy of the text (msv_fasta_read_device only)
};

namespace {

struct Dev {
    int prev = -1;
    bool ok = false;
    explicit Dev(int d) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(d) == hipSuccess;
    }
    ~Dev() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

msv_status hip_status(hipError_t e) {
    return e == hipErrorOutOfMemory ? MSV_ERR_OUT_OF_MEMORY : MSV_ERR_HIP;
}

#define FA_HIP(call)                               \
    do {                                           \
        hipError_t e_ = (call);                    \
        if (e_ != hipSuccess) return hip_status(e_); \
    } while (0)

template <typename T>
hipError_t dalloc(T*& p, uint64_t count) {
    return hipMalloc(reinterpret_cast<void**>(&p), std::max<uint64_t>(count, 1) * sizeof(T));
}

struct Scratch {
    uint2 *hs_ls = nullptr, *hs_ls_ex = nullptr, *pre_res = nullptr, *res = nullptr, *res_ex = nullptr;
    uint2 *rv = nullptr, *rv_ex = nullptr, *part = nullptr;
    fadev::TileCarry* carry = nullptr;
    fadev::Totals* tot = nullptr;
    uint32_t *rec_start = nullptr, *hdr_start = nullptr, *hdr_end = nullptr, *src = nullptr;
    uint8_t* bad = nullptr;
    ~Scratch() {
        for (void* p : {static_cast<void*>(hs_ls), static_cast<void*>(hs_ls_ex), static_cast<void*>(pre_res),
                        static_cast<void*>(res), static_cast<void*>(res_ex), static_cast<void*>(rv),
                        static_cast<void*>(rv_ex), static_cast<void*>(part), static_cast<void*>(carry),
                        static_cast<void*>(tot), static_cast<void*>(rec_start), static_cast<void*>(hdr_start),
                        static_cast<void*>(hdr_end), static_cast<void*>(src), static_cast<void*>(bad)})
            (void)hipFree(p);
    }
};

// Exclusive scan of n uint2 (3 launches); `part` holds >= ceil(n / 4096) elements.
template <int OPX, int OPY>
hipError_t scan_exclusive(const uint2* in, uint32_t n, uint2* out, uint2* part, hipStream_t st) {
    using namespace fadev;
    if (n == 0) return hipSuccess;
    const uint32_t np = (n + kTile - 1) / kTile;
    hipLaunchKernelGGL((scan_reduce<OPX, OPY>), dim3(np), dim3(kThreads), 0, st, in, n, part);
    hipLaunchKernelGGL((scan_partials<OPX, OPY>), dim3(1), dim3(kScanThreads), 0, st, part, np);
    hipLaunchKernelGGL((scan_down<OPX, OPY>), dim3(np), dim3(kThreads), 0, st, in, n, part, out);
    return hipGetLastError();
}

msv_status parse_on_device(msv_fasta_device* f, const uint8_t* d_text, uint64_t n, hipStream_t st) {
    using namespace fadev;
    if (n >= kMaxText) return MSV_ERR_INVALID_ARGUMENT;
    const uint32_t N = static_cast<uint32_t>(n);
    const uint32_t nt = std::max<uint32_t>(1, (N + kTileBytes - 1) / kTileBytes);
    const uint32_t tb = (nt + kThreads - 1) / kThreads;
    Scratch s;
    FA_HIP(dalloc(s.hs_ls, nt));
    FA_HIP(dalloc(s.hs_ls_ex, nt));
    FA_HIP(dalloc(s.pre_res, nt));
    FA_HIP(dalloc(s.res, nt));
    FA_HIP(dalloc(s.res_ex, nt));
    FA_HIP(dalloc(s.carry, nt));
    FA_HIP(dalloc(s.part, (nt + kTile - 1) / kTile));
    FA_HIP(dalloc(s.tot, 1));
    FA_HIP(hipMemsetAsync(s.tot, 0, sizeof(Totals), st));
    hipLaunchKernelGGL(fa_tile_summary, dim3(nt), dim3(kThreads), 0, st, d_text, N, s.hs_ls, s.pre_res);
    FA_HIP(hipGetLastError());
    FA_HIP((scan_exclusive<0, 1>(s.hs_ls, nt, s.hs_ls_ex, s.part, st)));
    hipLaunchKernelGGL(fa_tile_carry, dim3(tb), dim3(kThreads), 0, st, d_text, nt, s.hs_ls_ex, s.pre_res, s.res,
                       s.carry);
    FA_HIP(hipGetLastError());
    FA_HIP((scan_exclusive<0, 0>(s.res, nt, s.res_ex, s.part, st)));
    hipLaunchKernelGGL(fa_tile_rexcl, dim3(tb), dim3(kThreads), 0, st, nt, s.res_ex, s.carry);
    hipLaunchKernelGGL(fa_tile_totals, dim3(1), dim3(1), 0, st, nt, s.hs_ls, s.hs_ls_ex, s.res, s.res_ex, s.tot);
    FA_HIP(hipGetLastError());
    Totals tot{};
    FA_HIP(hipMemcpyAsync(&tot, s.tot, sizeof(Totals), hipMemcpyDeviceToHost, st));
    FA_HIP(hipStreamSynchronize(st));
    const uint32_t nrec = tot.headers, R = tot.residues;
    FA_HIP(dalloc(f->d_stage, R));
    FA_HIP(dalloc(s.rec_start, nrec));
    FA_HIP(dalloc(s.hdr_start, nrec));
    FA_HIP(dalloc(s.hdr_end, nrec));
    FA_HIP(dalloc(s.src, nrec));
    FA_HIP(dalloc(s.bad, nrec));
    FA_HIP(dalloc(s.rv, nrec));
    FA_HIP(dalloc(s.rv_ex, nrec));
    if ((nrec + kTile - 1) / kTile > (nt + kTile - 1) / kTile) {
        (void)hipFree(s.part);
        s.part = nullptr;
        FA_HIP(dalloc(s.part, (nrec + kTile - 1) / kTile));
    }
    FA_HIP(dalloc(f->d_offsets, static_cast<uint64_t>(nrec) + 1));
    FA_HIP(dalloc(f->d_spans, 2ull * nrec));
    FA_HIP(hipMemsetAsync(f->d_offsets, 0, sizeof(uint64_t), st));  // nrec == 0: offsets = {0}
    FA_HIP(hipMemsetAsync(s.hdr_end, 0xFF, std::max<uint32_t>(nrec, 1) * sizeof(uint32_t), st));
    FA_HIP(hipMemsetAsync(s.bad, 0, std::max<uint32_t>(nrec, 1), st));
    hipLaunchKernelGGL(fa_tile_emit, dim3(nt), dim3(kThreads), 0, st, d_text, N, s.carry, f->d_stage, s.rec_start,
                       s.hdr_start, s.hdr_end, s.bad, s.tot);
    FA_HIP(hipGetLastError());
    if (nrec) {
        const uint32_t rb = (nrec + kThreads - 1) / kThreads;
        hipLaunchKernelGGL(fa_rec_values, dim3(rb), dim3(kThreads), 0, st, nrec, s.rec_start, s.bad, s.tot, s.rv);
        FA_HIP(hipGetLastError());
        const uint32_t npr = (nrec + kTile - 1) / kTile;
        hipLaunchKernelGGL((scan_reduce<1, 1>), dim3(npr), dim3(kThreads), 0, st, s.rv, nrec, s.part);
        hipLaunchKernelGGL(fa_max_partials, dim3(1), dim3(kScanThreads), 0, st, s.part, npr, s.tot);
        FA_HIP((scan_exclusive<0, 0>(s.rv, nrec, s.rv_ex, s.part, st)));
        hipLaunchKernelGGL(fa_rec_write, dim3(rb), dim3(kThreads), 0, st, nrec, N, s.rv, s.rv_ex, s.rec_start,
                           s.hdr_start, s.hdr_end, f->d_offsets, f->d_spans, s.src, s.tot);
        FA_HIP(hipGetLastError());
    }
    FA_HIP(hipMemcpyAsync(&tot, s.tot, sizeof(Totals), hipMemcpyDeviceToHost, st));
    FA_HIP(hipStreamSynchronize(st));
    if (tot.error & 1u) return MSV_ERR_PARSE;
    f->count = tot.kept;
    f->rejected = nrec - tot.kept;
    f->residues = tot.kept_res;
    f->max_length = tot.max_len;
    f->d_codes = f->d_stage;
    if (f->rejected) {
        FA_HIP(dalloc(f->d_final, tot.kept_res));
        const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>(4096, (tot.kept + 3) / 4));
        hipLaunchKernelGGL(fa_compact, dim3(blocks), dim3(kThreads), 0, st, f->d_stage, tot.kept, f->d_offsets,
                           s.src, f->d_final);
        FA_HIP(hipGetLastError());
        FA_HIP(hipStreamSynchronize(st));
        f->d_codes = f->d_final;
    }
    return MSV_OK;
}

}  // namespace

extern "C" {

void msv_fasta_device_destroy(msv_fasta_device* f) {
    if (!f) return;
    Dev g(f->device);
    (void)hipFree(f->d_stage);
    (void)hipFree(f->d_final);
    (void)hipFree(f->d_offsets);
    (void)hipFree(f->d_spans);
    (void)hipFree(f->d_text);
    delete f;
}

msv_status msv_fasta_parse_device(int device, const uint8_t* d_text, uint64_t n, void* stream,
                                  msv_fasta_device** out) {
    if (!out || (n && !d_text)) return MSV_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    Dev g(device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    auto* f = new (std::nothrow) msv_fasta_device();
    if (!f) return MSV_ERR_OUT_OF_MEMORY;
    f->device = device;
    const msv_status s = parse_on_device(f, d_text, n, static_cast<hipStream_t>(stream));
    if (s != MSV_OK) {
        msv_fasta_device_destroy(f);
        return s;
    }
    *out = f;
    return MSV_OK;
}

msv_status msv_fasta_read_device(int device, const char* path, void* stream, msv_fasta_device** out) {
    if (!path || !out) return MSV_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    Dev g(device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    std::FILE* fp = std::fopen(path, "rb");
    if (!fp) return MSV_ERR_IO;
    std::fseek(fp, 0, SEEK_END);
    const long sz = std::ftell(fp);
    std::fseek(fp, 0, SEEK_SET);
    if (sz < 0) {
        std::fclose(fp);
        return MSV_ERR_IO;
    }
    const uint64_t n = static_cast<uint64_t>(sz);
    if (n >= fadev::kMaxText) {
        std::fclose(fp);
        return MSV_ERR_INVALID_ARGUMENT;
    }
    hipStream_t st = static_cast<hipStream_t>(stream);
    auto* f = new (std::nothrow) msv_fasta_device();
    if (!f) {
        std::fclose(fp);
        return MSV_ERR_OUT_OF_MEMORY;
    }
    f->device = device;
    // pinned staging in 64 MiB pieces: file read of piece k+1 overlaps the H2D copy of piece k
    constexpr uint64_t kPiece = 64ull << 20;
    uint8_t* pinned[2] = {nullptr, nullptr};
    hipEvent_t done[2] = {nullptr, nullptr};
    msv_status s = MSV_OK;
    if (dalloc(f->d_text, n) != hipSuccess) s = MSV_ERR_OUT_OF_MEMORY;
    for (int k = 0; k < 2 && s == MSV_OK; ++k) {
        if (hipHostMalloc(reinterpret_cast<void**>(&pinned[k]), std::min(kPiece, std::max<uint64_t>(n, 1))) !=
                hipSuccess ||
            hipEventCreateWithFlags(&done[k], hipEventDisableTiming) != hipSuccess)
            s = MSV_ERR_OUT_OF_MEMORY;
    }
    for (uint64_t off = 0, k = 0; s == MSV_OK && off < n; off += kPiece, ++k) {
        const uint64_t len = std::min(kPiece, n - off);
        uint8_t* buf = pinned[k & 1];
        if (k >= 2 && hipEventSynchronize(done[k & 1]) != hipSuccess) s = MSV_ERR_HIP;
        if (s == MSV_OK && std::fread(buf, 1, len, fp) != len) s = MSV_ERR_IO;
        if (s == MSV_OK && hipMemcpyAsync(f->d_text + off, buf, len, hipMemcpyHostToDevice, st) != hipSuccess)
            s = MSV_ERR_HIP;
        if (s == MSV_OK && hipEventRecord(done[k & 1], st) != hipSuccess) s = MSV_ERR_HIP;
    }
    std::fclose(fp);
    if (s == MSV_OK && hipStreamSynchronize(st) != hipSuccess) s = MSV_ERR_HIP;
    for (int k = 0; k < 2; ++k) {
        if (pinned[k]) (void)hipHostFree(pinned[k]);
        if (done[k]) (void)hipEventDestroy(done[k]);
    }
    if (s == MSV_OK) s = parse_on_device(f, f->d_text, n, st);
    if (s != MSV_OK) {
        msv_fasta_device_destroy(f);
        return s;
    }
    *out = f;
    return MSV_OK;
}

msv_status msv_fasta_device_download(const msv_fasta_device* f, uint8_t* codes, uint64_t* offsets, uint64_t* spans) {
    if (!f) return MSV_ERR_INVALID_ARGUMENT;
    Dev g(f->device);
    if (!g.ok) return MSV_ERR_NO_DEVICE;
    if (codes && f->residues) FA_HIP(hipMemcpy(codes, f->d_codes, f->residues, hipMemcpyDeviceToHost));
    if (offsets) FA_HIP(hipMemcpy(offsets, f->d_offsets, (f->count + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost));
    if (spans && f->count) FA_HIP(hipMemcpy(spans, f->d_spans, 2 * f->count * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return MSV_OK;
}

uint64_t msv_fasta_device_count(const msv_fasta_device* f) { return f ? f->count : 0; }
int msv_fasta_device_device(const msv_fasta_device* f) { return f ? f->device : -1; }
uint64_t msv_fasta_device_rejected(const msv_fasta_device* f) { return f ? f->rejected : 0; }
uint64_t msv_fasta_device_residues(const msv_fasta_device* f) { return f ? f->residues : 0; }
uint64_t msv_fasta_device_max_length(const msv_fasta_device* f) { return f ? f->max_length : 0; }
const uint8_t* msv_fasta_device_codes(const msv_fasta_device* f) { return f ? f->d_codes : nullptr; }
const uint64_t* msv_fasta_device_offsets(const msv_fasta_device* f) { return f ? f->d_offsets : nullptr; }
const uint64_t* msv_fasta_device_header_spans(const msv_fasta_device* f) { return f ? f->d_spans : nullptr; }
const uint8_t* msv_fasta_device_text(const msv_fasta_device* f) { return f ? f->d_text : nullptr; }

}  // extern "C"
