"""Seeded synthetic protein batches for benchmarks and tests.

Residues are uniform over the 20 amino acids, as FASTA_files/random_FASTA_generator.py:7-16
draws them, but seeded (the reference script is unseeded) and packed straight into the CSR code
stream the device consumes.  Lengths are uniform integers in [lmin, lmax].
"""
from __future__ import annotations

import numpy as np

AMINO_ACIDS = "ACDEFGHIKLMNPQRSTVWY"


def random_lengths(rng: np.random.Generator, n: int, lmin: int, lmax: int) -> np.ndarray:
    return rng.integers(lmin, lmax + 1, size=n, dtype=np.int64).astype(np.uint64)


def random_batch(seed: int, n: int, lmin: int, lmax: int) -> tuple[np.ndarray, np.ndarray]:
    """(codes uint8, offsets uint64[n+1]) with PCG64(seed)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    lengths = random_lengths(rng, n, lmin, lmax)
    offsets = np.zeros(n + 1, np.uint64)
    np.cumsum(lengths, out=offsets[1:])
    codes = rng.integers(0, 20, size=int(offsets[-1]), dtype=np.uint8)
    return codes, offsets


def write_fasta(path: str, codes: np.ndarray, offsets: np.ndarray, line: int = 70) -> None:
    """'> random i' headers, `line`-column residue lines (random_FASTA_generator.py:14-16)."""
    letters = np.frombuffer(AMINO_ACIDS.encode(), np.uint8)[codes].tobytes().decode()
    with open(path, "w") as f:
        for i in range(len(offsets) - 1):
            f.write(f"> random {i}\n")
            s = letters[int(offsets[i]):int(offsets[i + 1])]
            for k in range(0, len(s), line):
                f.write(s[k:k + line] + "\n")
