"""Irregular repeat-accumulate (IRA) codes with a DVB-S2-style structure.

BASELINE.json config 5 asks for "DVB-S2 n=64800 rate-1/2": that code is not
in the reference's matrix database, and the ETSI EN 302 307 address tables
are not available offline.  This module builds a code with the SAME
structure and size: n = 64800, k = 32400 (normal frame, rate 1/2); info
nodes in groups of 360 with 36 groups of degree 8 and 54 of degree 3 (the
standard's rate-1/2 degree profile, 226,799 edges in all); check degree 7;
parity part a staircase (dual diagonal), encoded by accumulation.  Only the
address table (which check rows a group's first bit reaches) is drawn from a
seeded RNG instead of the standard's table.  The resulting H has exactly the
standard's row and column weight profile, so decode cost and memory
behaviour are those of the real code; its waterfall is not pinned to the
real code's.

Column order is [info (k) | parity (m)]:
  bit j = 360*g + t of group g reaches rows (x + t*q) mod m for every table
  entry x of group g, q = m / 360 (DVB-S2's construction, ETSI EN 302 307
  section 5.3.2); parity p_r sits in rows r and r+1, so
  p_r = p_{r-1} xor (H_info u)_r  (p_{-1} = 0).
"""
import argparse

import numpy as np
from scipy import sparse

GROUP = 360


def ira_matrix(n, k, degrees, group=GROUP, seed=0):
    """H (CSR int32, m x n) of an IRA code.

    degrees: list of (n_groups, column degree) covering k/group info groups.
    Every residue class mod q (q = m/group) receives the same number of table
    entries, so every check row gets the same number of info edges.
    """
    m = n - k
    if k % group or m % group:
        raise ValueError("k and n-k must be multiples of the group size")
    q = m // group
    groups = [d for cnt, d in degrees for _ in range(cnt)]
    if len(groups) != k // group:
        raise ValueError(f"degree profile covers {len(groups)} groups, need {k // group}")
    total = sum(groups)
    if total % q:
        raise ValueError("table entries do not spread evenly over the residues mod q")
    rng = np.random.default_rng(seed)
    # residues: each class mod q exactly total/q times, no class twice in a
    # group -- every group takes the d classes with the most entries left
    # (random tie-break), largest groups first, which always completes
    left = np.full(q, total // q)
    table = [None] * len(groups)
    for g in sorted(range(len(groups)), key=lambda i: -groups[i]):
        d = groups[g]
        order = np.lexsort((rng.random(q), -left))
        res = order[:d]
        left[res] -= 1
        table[g] = res + q * rng.integers(0, group, size=d)
    rows, cols = [], []
    t = np.arange(group)
    for g, xs in enumerate(table):
        for x in xs:
            rows.append((x + t * q) % m)
            cols.append(g * group + t)
    # staircase parity: p_r in rows r and r+1
    r = np.arange(m)
    rows += [r, r[1:]]
    cols += [k + r, k + r[:-1]]
    rows = np.concatenate(rows)
    cols = np.concatenate(cols)
    H = sparse.csr_matrix((np.ones(len(rows), np.int32), (rows, cols)), shape=(m, n))
    H.sum_duplicates()
    if H.data.max() != 1:
        raise RuntimeError("duplicate edge in the IRA construction")
    H.sort_indices()
    return H


def dvbs2_profile_matrix(seed=0):
    """n=64800 rate-1/2 (normal frame) with DVB-S2's rate-1/2 degree profile."""
    return ira_matrix(64800, 32400, [(36, 8), (54, 3)], seed=seed)


def small_ira_matrix(seed=0):
    """n=1440 rate-1/2 with the same structure (group 36): fast tests."""
    return ira_matrix(1440, 720, [(8, 8), (12, 3)], group=36, seed=seed)


def is_ira(H):
    """True if H = [H_info | staircase] (what the on-device IRA encoder needs)."""
    H = sparse.csr_matrix(H)
    m, n = H.shape
    k = n - m
    P = H[:, k:].tocoo()
    want = set(zip(range(m), range(m))) | set(zip(range(1, m), range(m - 1)))
    return P.nnz == len(want) and set(zip(P.row.tolist(), P.col.tolist())) == want


def encode(H, u):
    """[B, k] info bits -> [B, n] codewords [u, p] of an IRA H (host helper)."""
    H = sparse.csr_matrix(H)
    m, n = H.shape
    k = n - m
    u = np.atleast_2d(np.asarray(u, dtype=np.int64))
    s = (H[:, :k] @ u.T).T % 2
    p = np.bitwise_xor.accumulate(s.astype(np.uint8), axis=1)
    return np.concatenate([u.astype(np.uint8), p], axis=1)


def main(argv=None):
    ap = argparse.ArgumentParser(description="write the DVB-S2-profile IRA code as an ALIST file")
    ap.add_argument("out")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--small", action="store_true", help="n=1440 test code instead of n=64800")
    a = ap.parse_args(argv)
    from .alist import write_alist
    H = small_ira_matrix(a.seed) if a.small else dvbs2_profile_matrix(a.seed)
    write_alist(H, a.out)
    print(f"{a.out}: {H.shape[0]} x {H.shape[1]}, {H.nnz} edges")


if __name__ == "__main__":
    main()
