#!/usr/bin/env python3
"""Regenerate the reference's own end-to-end test fixtures (tests/golden/e2e/).

Runs the reference's generators (project_tests/data_generation_scripts/
milestone{1..4}.py, read from /root/reference, never copied) at their default
size and seed (10,000 rows, seed 42; gen_all_for_staff_use.sh:9-13) and keeps
only their OUTPUTS: testNNgen.dsl (queries), testNNgen.exp (pandas-computed
expected output) and the CSV data they load. The load paths are written as
@DATA@/<file>.csv and substituted by tests/test_e2e.py.

pandas compatibility shim: the generators use
DataFrame.to_csv(line_terminator=...) and DataFrame.append, both removed from
pandas 2.x; they are mapped to lineterminator= and pd.concat.
"""
import os
import runpy
import shutil
import sys
import tempfile

import pandas as pd

REF = "/root/reference/project_tests/data_generation_scripts"
HERE = os.path.dirname(os.path.abspath(__file__))


def shim():
    orig_to_csv = pd.DataFrame.to_csv

    def to_csv(self, *a, **k):
        if "line_terminator" in k:
            k["lineterminator"] = k.pop("line_terminator")
        return orig_to_csv(self, *a, **k)

    def append(self, other, ignore_index=False, **k):
        return pd.concat([self, other if isinstance(other, pd.DataFrame) else pd.DataFrame([other])],
                         ignore_index=ignore_index)

    pd.DataFrame.to_csv = to_csv
    pd.DataFrame.append = append


def main():
    shim()
    out = tempfile.mkdtemp()
    sys.path.insert(0, REF)
    runs = [("milestone1.py", ["10000", "42", out, "@DATA@"]),
            ("milestone2.py", ["10000", "42", out, "@DATA@"]),
            ("milestone3.py", ["10000", "42", out, "@DATA@"]),
            ("milestone4.py", ["10000", "10000", "10000", "42", "1.0", "1000", out, "@DATA@"])]
    cwd = os.getcwd()
    os.chdir(REF)  # the scripts import data_gen_utils from their own directory
    try:
        for script, argv in runs:
            sys.argv = [script] + argv
            runpy.run_path(os.path.join(REF, script), run_name="__main__")
    finally:
        os.chdir(cwd)
    for f in sorted(os.listdir(out)):
        shutil.copy(os.path.join(out, f), os.path.join(HERE, f))
    shutil.rmtree(out)
    print("wrote", len(os.listdir(HERE)) - 1, "files to", HERE)


if __name__ == "__main__":
    main()
