"""Variant name -> the kernel symbol rocprofv3 reports for it (no GPU, no native library needed).

The library names its instantiations `msv_g<G>_s<S>[_a<SA>]_w<W>_p<PF>_d<D>` (csrc/msv_kernel.hip,
MSV_VARIANT / MSV_SPLIT_VARIANT); the kernel is `msvk::msv_batch_kernel<G, S, W, PF, BIG, D, SA, RPFO>`,
BIG = the table does not fit LDS (lds_rows_for < 21) and RPFO the residue prefetch of the zero-copy twin
that msv_score_batch runs on page-locked residues (0 for HBM-resident launches: bench.py's timed steps;
zero_copy_rpfo mirrors msv_kernel_impl.h zc_fn).
tools/rocprof_window.py and tools/pmc_summary.py filter dispatches on this exact symbol, and bench.py
publishes PMC traffic only when the committed PMC file names the kernel its timed steps run.
"""
from __future__ import annotations

import re

_LDS_LIMIT = 163840
_TABLE_ROWS = 21
_NAME = re.compile(r"^msv_g(\d+)_s(\d+)(?:_a(\d+))?_w(\d+)_p(\d+)_d(\d+)$")
_COOP = re.compile(r"^msv_coop_w(\d+)_s(\d+)(?:_a(\d+))?$")


def lds_rows_for(g: int, s: int) -> int:
    """msv_kernel.h lds_rows_for."""
    rows = _LDS_LIMIT // (g * s * 4)
    return _TABLE_ROWS if rows >= _TABLE_ROWS else rows


def parse_variant(name: str) -> dict:
    m = _NAME.match(name)
    if not m:
        raise ValueError(f"not an MSV variant name: {name!r}")
    g, s, sa, w, p, d = m.groups()
    g, s, w, p, d = int(g), int(s), int(w), int(p), int(d)
    sa = int(sa) if sa else 0
    big = sa == 0 and lds_rows_for(g, s) < _TABLE_ROWS
    return {"G": g, "S": s, "SA": sa, "waves": w, "PF": p, "D": d, "BIG": big}


def zero_copy_rpfo(v: dict) -> int:
    """The RPFO of the instantiation a launch reading page-locked residues in place runs (msv_kernel_impl.h
    zc_fn): 2 for 16/32-lane rows of more than 40 states (residues two rows ahead), kWideBlocks = 64 for
    rows of up to 40 states with 16+ lanes and PF <= 2 (64-row superblocks; buffers of >= 64 bytes), and 0
    -- no twin, the ordinary kernel -- for everything else (4/8-lane groups, whole-row rings, split,
    BIG and two-stream variants)."""
    plain = v["D"] == 1 and not v["BIG"] and v["SA"] == 0
    if plain and v["G"] in (16, 32) and v["S"] > 40:
        return 2
    if plain and v["G"] >= 16 and v["S"] <= 40 and v["PF"] <= 2:
        return 64
    return 0


def kernel_symbol(variant: str, zero_copy: bool = False) -> str:
    """`msv_batch_kernel<16, 88, 16, 2, false, 1, 0, 0>` for `msv_g16_s88_w16_p2_d1` (a substring of
    the demangled name rocprofv3 prints: `void msvk::msv_batch_kernel<...>(msvk::KernelArgs)`);
    `msv_coop_kernel<4, 6, 6>` for the cooperative plan `msv_coop_w4_s6` (msv_coop.hip), and
    `msv_coop_kernel<4, 10, 6>` for its split form `msv_coop_w4_s10_a6`."""
    m = _COOP.match(variant)
    if m:
        return f"msv_coop_kernel<{m.group(1)}, {m.group(2)}, {m.group(3) or m.group(2)}>"
    v = parse_variant(variant)
    rpfo = zero_copy_rpfo(v) if zero_copy else 0
    big = "true" if v["BIG"] else "false"
    return (f"msv_batch_kernel<{v['G']}, {v['S']}, {v['waves']}, {v['PF']}, {big}, {v['D']}, {v['SA']}, "
            f"{rpfo}>")
