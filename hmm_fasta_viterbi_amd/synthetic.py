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


# Amino-acid background frequencies in ACDEFGHIKLMNPQRSTVWY order: the reference's
# background_frequencies (algorithms/MSV_HMM.cpp:21-27, HMMER3's standard p7_bg for amino acids).
BACKGROUND = np.array([0.0787945, 0.0151600, 0.0535222, 0.0668298, 0.0397062, 0.0695071, 0.0229198,
                       0.0590092, 0.0594422, 0.0963728, 0.0237718, 0.0414386, 0.0482904, 0.0395639,
                       0.0540978, 0.0683364, 0.0540687, 0.0673417, 0.0114135, 0.0304133])


def background_batch(seed: int, n: int, length: int) -> tuple[np.ndarray, np.ndarray]:
    """n sequences of `length` residues drawn iid from BACKGROUND -- the null sequences HMMER3 scores to
    calibrate a profile's STATS LOCAL MSV mu (p7_MSVMu: L = 200, iid from the background)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    codes = rng.choice(20, size=n * length, p=BACKGROUND / BACKGROUND.sum()).astype(np.uint8)
    offsets = np.arange(0, n * length + 1, length, dtype=np.uint64)
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


def write_hmm(path: str, leng: int, seed: int) -> None:
    """A seeded HMMER3/b text profile of LENG `leng` (random -log probabilities in the ranges
    real Pfam profiles use), for model lengths beyond the reference's data/ set (max 2405).
    Layout as data/profile_HMMs/*.hmm: header tags, STATS LOCAL lines, COMPO block, then per node
    a match-emission line, an insert-emission line and a 7-field transition line ('*' = p 1)."""
    rng = np.random.Generator(np.random.PCG64(seed))

    def row(vals):
        return "".join(f"  {v:7.5f}" if v is not None else "        *" for v in vals)

    out = [
        "HMMER3/b [synthetic]",
        f"NAME  synthetic_{leng}_{seed}",
        f"LENG  {leng}",
        "ALPH  amino",
        "STATS LOCAL MSV       -9.9000  0.70000",
        "STATS LOCAL VITERBI  -10.5000  0.70000",
        "STATS LOCAL FORWARD   -4.0000  0.70000",
        "HMM     " + "".join(f"     {a}   " for a in AMINO_ACIDS),
        "            m->m     m->i     m->d     i->m     i->i     d->m     d->d",
    ]
    ins = rng.uniform(2.3, 4.5, 20)
    out.append("  COMPO " + row(rng.uniform(2.3, 4.5, 20)))
    out.append("        " + row(ins))
    out.append("        " + row([0.05, 4.1, 3.0, 0.62, 0.77, 0.0, None]))
    for k in range(1, leng + 1):
        out.append(f"{k:7d} " + row(rng.uniform(0.5, 5.5, 20)))
        out.append("        " + row(ins))
        last = k == leng
        out.append("        " + row([rng.uniform(0.01, 0.1), rng.uniform(3.5, 5.0),
                                     None if last else rng.uniform(4.0, 6.0), 0.62, 0.77,
                                     0.0 if last else rng.uniform(0.3, 0.6),
                                     None if last else rng.uniform(0.8, 1.2)]))
    out.append("//")
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")


def homolog_batch(match_emissions: np.ndarray, seed: int, n: int, lmin: int, lmax: int,
                  mutate: float = 0.1) -> tuple[np.ndarray, np.ndarray]:
    """Sequences EMITTED by the profile's match states (a run of consecutive states from a random
    start, each residue drawn from that state's match-emission distribution, a `mutate` fraction
    replaced by uniform residues), wrapped in uniform flanks.  They score far above random ones,
    so the DP's J state overtakes N (B = max(N, J) + move then depends on J) -- the rows the
    kernel's J-reduction path handles.  `match_emissions`: Profile_HMM.match_emissions, [M][20]
    with node 0 all zeros."""
    rng = np.random.Generator(np.random.PCG64(seed))
    probs = np.asarray(match_emissions, np.float64)[1:]
    leng = probs.shape[0]
    cdf = np.cumsum(probs / probs.sum(axis=1, keepdims=True), axis=1)
    seqs = []
    for _ in range(n):
        L = int(rng.integers(lmin, lmax + 1))
        core = min(L, leng, int(rng.integers(max(1, L // 2), L + 1)))
        start = int(rng.integers(0, leng - core + 1))
        u = rng.random(core)
        emitted = np.minimum((cdf[start:start + core] < u[:, None]).sum(axis=1), 19).astype(np.uint8)
        flip = rng.random(core) < mutate
        emitted[flip] = rng.integers(0, 20, size=int(flip.sum()), dtype=np.uint8)
        left = int(rng.integers(0, L - core + 1))
        seq = rng.integers(0, 20, size=L, dtype=np.uint8)
        seq[left:left + core] = emitted
        seqs.append(seq)
    offsets = np.zeros(n + 1, np.uint64)
    np.cumsum([len(s) for s in seqs], out=offsets[1:])
    codes = np.concatenate(seqs) if seqs else np.zeros(0, np.uint8)
    return codes, offsets


def gapped_homolog_batch(match_emissions: np.ndarray, seed: int, n: int, lmin: int, lmax: int,
                         p_delete: float = 0.03, max_delete: int = 60, p_insert: float = 0.03,
                         max_insert: int = 8, mutate: float = 0.05) -> tuple[np.ndarray, np.ndarray]:
    """Sequences emitted along a profile path WITH gaps: from a random start node, each step either emits
    from the current match state, skips a run of 1..max_delete nodes (a deletion: the Viterbi path goes
    through D states, often across the 64-lane kernel's lane boundaries), or emits 1..max_insert uniform
    residues (an insertion: I states); uniform flanks around the core.  These are the sequences whose best
    Viterbi path uses I and D states, which homolog_batch's ungapped cores never do."""
    rng = np.random.Generator(np.random.PCG64(seed))
    probs = np.asarray(match_emissions, np.float64)[1:]
    leng = probs.shape[0]
    cdf = np.cumsum(probs / probs.sum(axis=1, keepdims=True), axis=1)
    seqs = []
    for _ in range(n):
        L = int(rng.integers(lmin, lmax + 1))
        core_target = int(rng.integers(max(1, L // 2), L + 1))
        k = int(rng.integers(0, max(1, leng // 3)))
        core = []
        while k < leng and len(core) < core_target:
            u = rng.random()
            if u < p_delete:
                k += int(rng.integers(1, max_delete + 1))
                continue
            if u < p_delete + p_insert:
                core.extend(rng.integers(0, 20, size=int(rng.integers(1, max_insert + 1))).tolist())
            x = int(min((cdf[k] < rng.random()).sum(), 19))
            core.append(int(rng.integers(0, 20)) if rng.random() < mutate else x)
            k += 1
        core = np.array(core[:L], np.uint8)
        left = int(rng.integers(0, L - len(core) + 1))
        seq = rng.integers(0, 20, size=L, dtype=np.uint8)
        seq[left:left + len(core)] = core
        seqs.append(seq)
    offsets = np.zeros(n + 1, np.uint64)
    np.cumsum([len(s) for s in seqs], out=offsets[1:])
    codes = np.concatenate(seqs) if seqs else np.zeros(0, np.uint8)
    return codes, offsets


def concat_batches(*batches: tuple[np.ndarray, np.ndarray]) -> tuple[np.ndarray, np.ndarray]:
    """Concatenate CSR batches (codes, offsets) in order."""
    codes = np.concatenate([c for c, _ in batches])
    lens = np.concatenate([np.diff(o) for _, o in batches]).astype(np.uint64)
    offsets = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(lens, out=offsets[1:])
    return codes, offsets
