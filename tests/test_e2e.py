"""End-to-end drop-in: the reference's own server, linked against libmq.so, replays
the reference's own DSL test suite (tests 1-37, milestones 1-4).

Binaries (oracle/Makefile, from /root/reference/src as shipped; they travel to the
GPU box prebuilt in oracle/_ref/):
  server_ref  server.o parse.o utils.o db_manager.o client_context.o query.o multimap.o index.o
  server_mq   the same objects with query.o multimap.o replaced by libmq.so
  client      client.o utils.o

The harness mirrors infra_scripts/test_milestone.sh (one server, restarted before
tests 2, 5, 11, 19, 20, 29, 32 to exercise persistence) and
infra_scripts/verify_output_standalone.sh (strip comments and whitespace, print
decimals as %0.2f, diff, and on mismatch diff the numerically sorted files).

  * CPU test: server_ref passes the suite as the survey recorded it (fixtures and
    harness are sound; the reference's own failures are listed in REF_FAILS).
  * GPU test: server_mq passes every test the reference passes, plus test 14 (the
    reference prints an unterminated buffer for an empty result, query.c:253), and
    its normalised output equals the reference server's, test by test.
"""
import os
import re
import shutil
import signal
import socket
import subprocess
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
E2E = os.path.join(ROOT, "tests", "golden", "e2e")
REFBIN = os.path.join(ROOT, "oracle", "_ref")
TESTS = list(range(1, 38))
RESTART_BEFORE = {2, 5, 11, 19, 20, 29, 32}           # test_milestone.sh:64-75
# Reference failures recorded in SURVEY.md §4: 14 (print of an empty result),
# 25 (index build leaves stale positions, index.c:152-178; index.o is linked into
# both servers, so it fails for server_mq as well).
REF_FAILS = {14, 25}
SOCK = "mq_e2e.sock"


def _have(name):
    return os.path.exists(os.path.join(REFBIN, name))


def normalise(text: str) -> list:
    """verify_output_standalone.sh:20-30."""
    out = []
    for line in text.splitlines():
        line = re.sub(r"\x1B\[([0-9]{1,2}(;[0-9]{1,2})?)?[m|K]", "", line)
        line = re.sub(r"--.*$", "", line).strip()
        if not line:
            continue
        fields = []
        for f in line.split(","):
            if "." in f:
                try:
                    f = "%0.2f" % float(f)
                except ValueError:
                    pass
            fields.append(f)
        out.append(",".join(fields))
    return out


def _ws(lines):
    return [re.sub(r"\s+", " ", l).strip() for l in lines if l.strip()]


def _sortkey(line):
    m = re.match(r"\s*(-?\d+(\.\d+)?)", line)
    return (0, float(m.group(1)), line) if m else (1, 0.0, line)


def verdict(out_lines, exp_lines) -> str:
    a, b = _ws(out_lines), _ws(exp_lines)
    if a == b:
        return "pass"
    if sorted(a, key=_sortkey) == sorted(b, key=_sortkey):
        return "pass-sorted"
    return "fail"


class Server:
    def __init__(self, binary, workdir, log):
        self.binary, self.workdir, self.log = binary, workdir, log
        self.proc = None

    def start(self):
        sock = os.path.join(self.workdir, SOCK)
        if os.path.exists(sock):
            os.unlink(sock)
        self.proc = subprocess.Popen([self.binary], cwd=self.workdir, stdout=self.log,
                                     stderr=subprocess.STDOUT, start_new_session=True)
        deadline = time.time() + 60
        while time.time() < deadline:
            if self.proc.poll() is not None:
                raise RuntimeError(f"{self.binary} exited early ({self.proc.returncode})")
            if os.path.exists(sock):
                try:
                    with socket.socket(socket.AF_UNIX) as s:
                        s.connect(sock)
                    return
                except OSError:
                    pass
            time.sleep(0.05)
        raise RuntimeError(f"{self.binary} did not open {SOCK}")

    def stop(self):
        if self.proc and self.proc.poll() is None:
            os.killpg(self.proc.pid, signal.SIGKILL)
            self.proc.wait(timeout=30)
        self.proc = None


def run_dsl_files(server_bin: str, workdir: str, names) -> dict:
    """Replay DSL files from tests/golden/e2e in ONE server session (no restart):
    {name: normalised output lines}."""
    os.makedirs(workdir, exist_ok=True)
    for f in os.listdir(E2E):
        if f.endswith(".csv"):
            shutil.copy(os.path.join(E2E, f), workdir)
    log = open(os.path.join(workdir, "server.log"), "ab")
    srv = Server(server_bin, workdir, log)
    out = {}
    try:
        srv.start()
        for name in names:
            dsl = open(os.path.join(E2E, name)).read().replace("@DATA@", ".")
            cp = subprocess.run([os.path.join(REFBIN, "client")], input=dsl.encode(), cwd=workdir,
                                capture_output=True, timeout=600)
            out[name] = normalise(cp.stdout.decode(errors="replace"))
    finally:
        srv.stop()
        log.close()
    return out


def run_suite(server_bin: str, workdir: str, tests=TESTS) -> dict:
    """Returns {test_id: (normalised output lines, verdict)}."""
    os.makedirs(workdir, exist_ok=True)
    for f in os.listdir(E2E):
        if f.endswith(".csv"):
            shutil.copy(os.path.join(E2E, f), workdir)
    log = open(os.path.join(workdir, "server.log"), "ab")
    srv = Server(server_bin, workdir, log)
    results = {}
    try:
        for i, tid in enumerate(tests):
            print(f"{os.path.basename(server_bin)}: test {tid}", flush=True)  # progress (pytest -s)
            if i == 0 or tid in RESTART_BEFORE or srv.proc is None or srv.proc.poll() is not None:
                srv.stop()
                srv.start()
            dsl = open(os.path.join(E2E, f"test{tid:02d}gen.dsl")).read().replace("@DATA@", ".")
            exp = open(os.path.join(E2E, f"test{tid:02d}gen.exp")).read()
            cp = subprocess.run([os.path.join(REFBIN, "client")], input=dsl.encode(), cwd=workdir,
                                capture_output=True, timeout=600)
            out = normalise(cp.stdout.decode(errors="replace"))
            results[tid] = (out, verdict(out, normalise(exp)))
    finally:
        srv.stop()
        log.close()
    return results


needs_bins = pytest.mark.skipif(not (_have("server_ref") and _have("client")),
                                reason="oracle/_ref server/client not built (needs /root/reference)")


@needs_bins
@pytest.mark.timeout(900)
def test_reference_server_passes_its_suite(tmp_path):
    res = run_suite(os.path.join(REFBIN, "server_ref"), str(tmp_path))
    failed = sorted(t for t, (_, v) in res.items() if v == "fail")
    assert set(failed) <= REF_FAILS, f"reference server failed {failed}"


@pytest.mark.gpu
@needs_bins
@pytest.mark.skipif(not _have("server_mq"), reason="server_mq not built")
@pytest.mark.timeout(900)
def test_libmq_dropin_server_passes_suite_and_matches_reference(tmp_path):
    mine = run_suite(os.path.join(REFBIN, "server_mq"), str(tmp_path / "mq"))
    ref = run_suite(os.path.join(REFBIN, "server_ref"), str(tmp_path / "ref"))
    failed = sorted(t for t, (_, v) in mine.items() if v == "fail")
    assert set(failed) <= {25}, f"server_mq failed {failed}"
    differ = [t for t in TESTS if t not in REF_FAILS and _ws(mine[t][0]) != _ws(ref[t][0])]
    assert not differ, f"server_mq output differs from the reference server on tests {differ}"
    # every INT print through the GPU formatter (mq_format_int32), not just >= 32768 tuples
    os.environ["MQ_PRINT_GPU_MIN"] = "1"
    try:
        gpu_print = run_suite(os.path.join(REFBIN, "server_mq"), str(tmp_path / "mq_gpu_print"))
    finally:
        del os.environ["MQ_PRINT_GPU_MIN"]
    differ = [t for t in TESTS if _ws(gpu_print[t][0]) != _ws(mine[t][0])]
    assert not differ, f"GPU-formatted print differs on tests {differ}"


@pytest.mark.gpu
@needs_bins
@pytest.mark.skipif(not _have("server_mq_ix"), reason="server_mq_ix not built")
@pytest.mark.timeout(900)
def test_libmq_dropin_with_gpu_index_build(tmp_path):
    """server_mq_ix also links libmq's build_index (GPU sort in the reference
    quicksort's own order of equal values). Its verdicts must be the reference's and
    its output the reference server's, line for line (tests 21, 22, 29 index columns
    with equal values)."""
    mine = run_suite(os.path.join(REFBIN, "server_mq_ix"), str(tmp_path / "mqix"))
    ref = run_suite(os.path.join(REFBIN, "server_ref"), str(tmp_path / "ref"))
    failed = sorted(t for t, (_, v) in mine.items() if v == "fail")
    assert set(failed) <= {25}, f"server_mq_ix failed {failed}"
    differ = [t for t in TESTS if t not in REF_FAILS and _ws(mine[t][0]) != _ws(ref[t][0])]
    assert not differ, f"server_mq_ix output differs from the reference server on tests {differ}"


@needs_bins
@pytest.mark.timeout(300)
def test_reference_server_residency_dsl(tmp_path):
    """The residency DSL is meaningful on the reference: it prints every query."""
    out = run_dsl_files(os.path.join(REFBIN, "server_ref"), str(tmp_path), [RESIDENCY_DSL])
    assert len(out[RESIDENCY_DSL]) > 20


RESIDENCY_DSL = "residency_noshutdown.dsl"


@pytest.mark.gpu
@needs_bins
@pytest.mark.parametrize("binary", ["server_mq", "server_mq_ix"])
@pytest.mark.timeout(300)
def test_load_index_query_same_session(tmp_path, binary):
    """load_db keeps the columns resident in HBM, then the index
    build rewrites the other columns in place (reference build_index in server_mq,
    libmq's in server_mq_ix), then select/fetch/sum on them in the same session.
    The output must be the reference server's, line for line."""
    if not _have(binary):
        pytest.skip(f"{binary} not built")
    mine = run_dsl_files(os.path.join(REFBIN, binary), str(tmp_path / "mq"), [RESIDENCY_DSL])
    ref = run_dsl_files(os.path.join(REFBIN, "server_ref"), str(tmp_path / "ref"), [RESIDENCY_DSL])
    assert _ws(mine[RESIDENCY_DSL]) == _ws(ref[RESIDENCY_DSL])
