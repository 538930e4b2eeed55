"""CSV inputs for the load path (db_manager.c:240-322 load_db) — shared by the golden
generator (tests/golden/make_csv_goldens.py), the CPU oracle tests and the GPU
parity tests. Every case is deterministic: (name, ncols, data bytes). The data is
what load_db reads after its header line.
"""
from __future__ import annotations

import numpy as np


def _long_lines() -> bytes:
    out = []
    for L in (1021, 1022, 1023, 1024, 1025, 2045, 2046, 2047, 2048, 3070, 5000):
        # L bytes before the '\n': a run of "12345," cells, cut at L
        body = (b"12345," * (L // 6 + 2))[:L]
        out.append(body + b"\n")
        out.append(b"7,8,9\n")
    # a long line of spaces then a number straddling a 1023-byte piece boundary
    out.append(b" " * 1020 + b"123456,42\n")
    out.append(b"-" + b"0" * 1500 + b"17,3\n")
    return b"".join(out)


def _random_text(rng, nbytes: int, alphabet: bytes) -> bytes:
    a = np.frombuffer(alphabet, dtype=np.uint8)
    return a[rng.integers(0, len(a), nbytes)].tobytes()


def _random_csv(rng, rows: int, ncols: int, lo: int, hi: int) -> bytes:
    vals = rng.integers(lo, hi, size=(rows, ncols), dtype=np.int64)
    return b"".join((",".join(str(int(v)) for v in r) + "\n").encode() for r in vals)


def cases() -> list[tuple[str, int, bytes]]:
    rng = np.random.default_rng(20261016)
    c = []
    c.append(("basic", 3, b"1,2,3\n4,5,6\n-7,-8,-9\n"))
    c.append(("empty", 2, b""))
    c.append(("one_no_newline", 1, b"42"))
    c.append(("blank_lines", 2, b"\n\n5,6\n\n\n"))
    c.append(("whitespace_signs", 4,
              b" 1,\t2 ,+3,-4\n\v\f\r5,  -6,+-7,- 8\n9x,0x1F,1e5,--3\n"
              b"12\r\n34 ,56\r\n"))
    c.append(("overflow", 3,
              b"2147483647,2147483648,-2147483648\n"
              b"-2147483649,4294967295,4294967296\n"
              b"9223372036854775807,9223372036854775808,-9223372036854775808\n"
              b"-9223372036854775809,99999999999999999999,-99999999999999999999\n"
              b"0000000000000000000000000123,-0000000000000000000000000000042,18446744073709551616\n"
              b"1234567890123456789,12345678901234567890,-1234567890123456789\n"))
    c.append(("missing_extra", 4,
              b"1,2,3,4\n5\n6,7\n8,9,10,11,12,13\n,\n,,,,\n14,,15\n\n16,17,18\n"))
    c.append(("missing_first_row", 3, b"1\n2,3\n4,5,6\n7\n"))
    c.append(("zero_cols_in_text", 2, b"abc\n,\n"))
    c.append(("nul_bytes", 3, b"1,2\x003\n4,5,6\n\x007,8,9\n10,\x0011,12\n"))
    c.append(("long_lines", 3, _long_lines()))
    c.append(("long_only", 2, b"9," * 2000 + b"\n"))
    c.append(("long_no_newline", 1, b"5" + b" " * 3000))
    c.append(("trailing_long_newline", 2, b"1,2\n" + b"3" * 1022 + b"\n" + b"4," * 700))
    c.append(("fuzz_small", 3, _random_text(rng, 20000, b"0123456789-+ ,\n\t\r")))
    c.append(("fuzz_sparse_newlines", 5, _random_text(rng, 60000, b"0123456789" * 20 + b",,-\n")))
    c.append(("fuzz_nul", 2, _random_text(rng, 30000, b"0123456789,\n\x00 ")))
    c.append(("random_4col", 4, _random_csv(rng, 20000, 4, -2**31, 2**31)))
    c.append(("random_1col", 1, _random_csv(rng, 50000, 1, 0, 10**9)))
    c.append(("wide_12col", 12, _random_csv(rng, 3000, 12, -1000, 1000)))
    c.append(("wide_missing", 10, b"".join(
        (",".join(str(v) for v in range(int(k))) + "\n").encode()
        for k in rng.integers(0, 14, 4000))))
    return c


def token_counts(data: bytes) -> list[int]:
    """Tokens strsep finds in each fgets(line, 1024) piece of `data` (a NUL ends the
    string; db_manager.c:306-311) — used to mark the cells the reference leaves
    uninitialised: column j before the first row that has a token j."""
    counts, at, n = [], 0, len(data)
    while at < n:
        nl = data.find(b"\n", at, at + 1023)
        end = min(at + 1023, n) if nl < 0 else nl + 1
        piece = data[at:end].split(b"\x00", 1)[0]
        counts.append(piece.count(b",") + 1)
        at = end
    return counts


def leading_unset(data: bytes, ncols: int) -> list[int]:
    """Per column, the rows before the first row with that token (their value is
    the reference's uninitialised row[] slot)."""
    counts = token_counts(data)
    lead = []
    for j in range(ncols):
        r = next((i for i, c in enumerate(counts) if c > j), len(counts))
        lead.append(r)
    return lead
