"""Index-build inputs and the build_index model — shared by the golden generator
(tests/golden/make_index_goldens.py), the CPU oracle tests and the GPU tests.

A case is (name, columns int32[ncols][n], spec) with spec a list of (column,
clustered) as create(idx, ...) declares them (db_manager.c:154-162).
model() composes the oracle's restatement of the reference quicksort (oracle/refcpu.c
rc_index_build_lomuto, equal values in the reference's own order) exactly as
build_index (src/index.c:152-178) does: columns in order; clustered -> sorted values,
positions 0..n-1, every other column reordered by the permutation; unclustered ->
sorted values, the permutation, the 100-bin histogram. Parity is exact: no
canonicalisation of equal values.
"""
from __future__ import annotations

import numpy as np

BIN_NUM = 100


def cases() -> list:
    rng = np.random.default_rng(20261017)
    out = []
    n = 3000
    out.append(("distinct_clustered", np.stack([rng.permutation(n), rng.integers(-10**6, 10**6, n),
                                                rng.integers(0, 10**9, n)]).astype(np.int32), [(0, True)]))
    out.append(("distinct_unclustered", np.stack([rng.permutation(n) * 7 - 9000,
                                                  rng.integers(0, 50, n)]).astype(np.int32), [(0, False)]))
    out.append(("dups_unclustered", np.stack([rng.integers(0, 200, 2000), rng.integers(0, 9, 2000)])
                .astype(np.int32), [(0, False)]))
    out.append(("clustered_then_unclustered_dups",
                np.stack([rng.integers(-500, 500, 2500), rng.permutation(2500),
                          rng.integers(0, 400, 2500)]).astype(np.int32), [(1, True), (2, False)]))
    out.append(("unclustered_then_clustered",
                np.stack([rng.permutation(2000), rng.integers(0, 30, 2000),
                          rng.integers(-99, 99, 2000)]).astype(np.int32), [(0, False), (1, True)]))
    out.append(("negatives_wide", np.stack([rng.integers(-10**9, 10**9, 3000),
                                            rng.integers(0, 5, 3000)]).astype(np.int32), [(0, False)]))
    out.append(("small_range_bins", np.stack([rng.integers(7, 7 + 100, 1500),
                                              rng.integers(0, 3, 1500)]).astype(np.int32), [(0, False)]))
    # (an unclustered index on a column spanning < 99 values divides by zero in the
    # reference's build_histogram, index.c:65,78: no such case can be pinned)
    return out


def csv_text(cols: np.ndarray) -> bytes:
    hdr = ",".join(f"db.tbl.c{j}" for j in range(len(cols))) + "\n"
    return (hdr + "".join(",".join(str(int(v)) for v in row) + "\n" for row in cols.T)).encode()


def hist_params(col: np.ndarray):
    """insert_row's min/max, then build_histogram's bin_size and bin values."""
    mn, mx = int(col.min()), int(col.max())
    d = int(np.int32(np.int64(mx) - mn))  # int arithmetic of the reference (wraps)
    bin_size = (abs(d) // (BIN_NUM - 1)) * (1 if d >= 0 else -1)  # C truncates toward 0
    start = np.uint64(0)
    values = []
    for _ in range(BIN_NUM):
        values.append(int(np.int32(np.uint32(int(start) & 0xFFFFFFFF))))
        start = np.uint64((int(start) + (bin_size & 0xFFFFFFFFFFFFFFFF)) & 0xFFFFFFFFFFFFFFFF)
    return mn, bin_size, values


def model(refcpu, cols: np.ndarray, spec) -> dict:
    cols = cols.copy()
    out = {}
    for j, clustered in spec:
        v, p = refcpu.index_build_lomuto(cols[j])
        out[f"ix{j}_values"] = v
        if clustered:
            out[f"ix{j}_positions"] = np.arange(len(v), dtype=np.uint64)
            for o in range(len(cols)):
                if o != j:
                    cols[o] = cols[o][p.astype(np.int64)]
        else:
            out[f"ix{j}_positions"] = p
            mn, bin_size, values = hist_params(cols[j])
            out[f"hist{j}_bin_size"] = bin_size
            out[f"hist{j}_values"] = np.array(values, dtype=np.int64)
            out[f"hist{j}_counts"] = refcpu.histogram(cols[j], mn, bin_size)[:BIN_NUM]
    out["cols"] = cols
    return out
