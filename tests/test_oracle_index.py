"""Pin the index-build restatement (oracle/refcpu.c rc_index_build_lomuto /
rc_histogram, composed as build_index in tests/indexcases.py model()) against the
reference's own build_index (tests/golden/index_goldens.json, from
oracle/_ref/libdbm.so) and its own quicksort symbol: exact, equal values included.
CPU only.
"""
import json
import os

import numpy as np
import pytest

from indexcases import cases, csv_text, model

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
    got = digest(refcpu, result, spec)
    for k, v in got.items():
        assert v == g[k], (name, k)


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


def _lomuto_inputs():
    rng = np.random.default_rng(11)
    yield "empty", np.zeros(0, np.int32)
    yield "one", np.array([5], np.int32)
    yield "all_equal", np.full(700, 3, np.int32)
    yield "sorted", np.arange(900, dtype=np.int32)
    yield "reverse", np.arange(900, 0, -1).astype(np.int32)
    yield "two_values", rng.integers(0, 2, 1500).astype(np.int32)
    yield "few_values", rng.integers(-3, 4, 2000).astype(np.int32)
    yield "dups", rng.integers(0, 200, 3000).astype(np.int32)
    yield "distinct", rng.permutation(3000).astype(np.int32)
    yield "extremes", rng.choice(np.array([-2**31, 2**31 - 1, 0, -1, 1], np.int32), 1200)
    yield "sorted_dups", np.sort(rng.integers(0, 50, 1000)).astype(np.int32)
    yield "organ_pipe", np.concatenate([np.arange(500), np.arange(500, 0, -1)]).astype(np.int32)


@pytest.mark.parametrize("name,col", list(_lomuto_inputs()))
def test_lomuto_restatement_equals_reference_quicksort(refcpu, name, col):
    """rc_index_build_lomuto against the reference's own quicksort symbol (libdbm.so):
    values AND positions identical, equal values included."""
    import refload
    if not refload.have():
        pytest.skip("oracle/_ref/libdbm.so not built (no /root/reference)")
    rv, rp = refload.quicksort(col)
    v, p = refcpu.index_build_lomuto(col)
    assert np.array_equal(v, rv), name
    assert np.array_equal(p, rp), name


def _qs_goldens():
    import json
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "quicksort_goldens.json")
    return [c for c in json.load(open(path)) if c["log2n"] == 22]


@pytest.mark.parametrize("case", _qs_goldens(), ids=lambda c: f"s{c['seed']}_m{c['modulus']}")
def test_lomuto_restatement_2e22_vs_reference_quicksort(refcpu, case):
    """rc_index_build_lomuto (the iterative restatement the GPU
    tests compare with) against the reference's own quicksort at 2^22 rows: the
    goldens that symbol produced (make_quicksort_goldens.py) and, where libdbm.so is
    built, a fresh run of the symbol itself on the seed-42 column."""
    n = case["n"]
    col = refcpu.gen_uniform(n, case["seed"], case["modulus"])
    assert f"{refcpu.fnv1a64(col):016x}" == case["col_fnv"]
    v, p = refcpu.index_build_lomuto(col)
    assert f"{refcpu.fnv1a64(v):016x}" == case["values_fnv"]
    assert f"{refcpu.fnv1a64(p):016x}" == case["positions_fnv"]
    assert int(np.count_nonzero(v[1:] == v[:-1])) == case["ties"]
    import refload
    if case["seed"] == 42 and refload.have():
        rv, rp = refload.quicksort(col)
        assert np.array_equal(v, rv) and np.array_equal(p, rp)
