"""Pin the index-build restatement (oracle/refcpu.c rc_index_build / rc_histogram,
composed as build_index in tests/indexcases.py model()) against the reference's own
build_index (tests/golden/index_goldens.json, from oracle/_ref/libdbm.so).

The reference's quicksort decides the order of equal values by itself, so the
comparison is on canon(): exact sorted values, histogram and, within each run of
equal indexed values, the sorted positions / reordered rows. Where the reference's
raw positions are already canonical (distinct values), the restatement's raw output
must equal them too. CPU only.
"""
import json
import os

import numpy as np
import pytest

from indexcases import canon, cases, csv_text, model

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "index_goldens.json")))
CASES = {name: (cols, spec) for name, cols, spec in cases()}


def digest(refcpu, c, spec):
    f = lambda x: f"{refcpu.fnv1a64(np.ascontiguousarray(x)):016x}"  # noqa: E731
    d = {"cols": [f(col.astype(np.int32)) for col in c["cols"]]}
    for j, clustered in spec:
        d[f"ix{j}_values"] = f(np.asarray(c[f"ix{j}_values"], dtype=np.int32))
        d[f"ix{j}_positions"] = f(np.asarray(c[f"ix{j}_positions"], dtype=np.uint64))
        if not clustered:
            d[f"hist{j}_bin_size"] = int(c[f"hist{j}_bin_size"])
            d[f"hist{j}_values"] = [int(v) for v in c[f"hist{j}_values"]]
            d[f"hist{j}_counts"] = [int(v) for v in c[f"hist{j}_counts"]]
    return d


def check_index_result(refcpu, name, result):
    """result: a build_index outcome (cols + ix*/hist* arrays) for case `name`."""
    g = GOLD[name]
    spec = [tuple(x) for x in g["spec"]]
    got = digest(refcpu, canon(result, spec), spec)
    for k, v in got.items():
        assert v == g[k], (name, k)
    raw = digest(refcpu, result, spec)
    for j, exact in g["exact_positions"].items():
        if exact:
            assert raw[f"ix{j}_positions"] == g[f"ix{j}_positions"], (name, j)


def test_index_inputs_match_goldens(refcpu):
    assert set(CASES) == set(GOLD)
    for name, (cols, spec) in CASES.items():
        assert f"{refcpu.fnv1a64_bytes(csv_text(cols)):016x}" == GOLD[name]["in_fnv"], name
        assert [tuple(x) for x in GOLD[name]["spec"]] == [tuple(x) for x in spec]


@pytest.mark.parametrize("name", sorted(CASES))
def test_index_restatement_vs_reference_goldens(refcpu, name):
    cols, spec = CASES[name]
    check_index_result(refcpu, name, model(refcpu, cols, spec))


def test_index_restatement_is_stable(refcpu):
    rng = np.random.default_rng(3)
    col = rng.integers(-5, 5, 10_000).astype(np.int32)
    v, p = refcpu.index_build(col)
    assert np.array_equal(v, np.sort(col, kind="stable"))
    assert np.array_equal(p, np.argsort(col, kind="stable").astype(np.uint64))
