"""Range query on the CPU: the product kernels
(k_query_match, k_query_stream, the decoder's kernels in csrc/vcfc_decode.hip)
and the host driver (vcfc_dec::query_section) compiled against the fiber SIMT
emulator, checked against the reference CLI's own query outputs
(tests/golden/query_cases.json) and against the oracle on valid and mutated
inputs.  test_gpu_query.py repeats these on the GPU."""
import hashlib

import pytest

import decode_cases as D
import emu_io as E
import golden_io as G

OK, E_FORMAT = 0, 8


def check(data, q, name=""):
    pq = G.oracle_parse_query(q)
    assert pq is not None, q
    st_o, want = G.oracle_query(data, q)
    st, got = E.emu_query(data, *pq, out_batch=1 << 12)
    assert st == (OK if st_o == 0 else E_FORMAT), (name, q, st, st_o)
    assert got == want, (name, q, len(got), len(want))
    return st, got


def test_reference_cli_cases():
    n = 0
    for c, data in G.query_cases():
        q = c["query"].encode()
        if c["rc"] == 1:   # the query string does not parse: the reference exits before reading the file
            assert G.oracle_parse_query(q) is None
            continue
        st, got = check(data, q, c["file"])
        if c["rc"] == 0:
            assert st == OK and hashlib.sha256(got).hexdigest() == c["stdout_sha256"], (c, len(got))
        else:   # the reference aborts and loses its unflushed stdout: what it printed is a prefix
            assert st == E_FORMAT
            assert hashlib.sha256(got[:c["stdout_len"]]).hexdigest() == c["stdout_sha256"], c
        n += 1
    assert n >= 20


@pytest.mark.parametrize("seed", [1, 2])
def test_query_files_match_oracle(seed):
    for name, data, qs in D.query_files(seed):
        for q in qs:
            check(data, q, name)


def test_mutated_decode_files_match_oracle():
    for name, data in D.mutated_files(5):
        for q in (b"22", b"22:110-120"):
            check(data, q, name)
