"""Decoder on the CPU: the product kernels
(csrc/vcfc_decode.hip) and host driver (csrc/vcfc_decode_driver.h) compiled
against the fiber SIMT emulator, checked byte-exact against the reference's
own decompress outputs (tests/golden) and against the oracle on valid and
mutated inputs.  test_gpu_decode.py repeats these on the GPU."""
import pytest

import decode_cases as D
import emu_io as E
import golden_io as G

OK, E_FORMAT = 0, 8


def check(data, name=""):
    st_o, want = G.oracle_decompress(data, cap=len(data) * 600 + 4096)
    st, got = E.emu_decompress(data, out_batch=1 << 12)
    assert st == (OK if st_o == 0 else E_FORMAT), (name, st, st_o)
    assert got == want, (name, len(got), len(want))


def test_reference_round_trip_config1():
    st, dec = E.emu_decompress(G.gz("random_100x10000.vcfc.gz"), out_batch=1 << 20)
    assert st == OK and dec == G.gz("random_100x10000.vcf.gz")


def test_reference_fuzz_decode_corpus():
    st, dec = E.emu_decompress(G.gz("fuzz_decode.vcfc.gz"), out_batch=1 << 16)
    assert st == OK and dec == G.gz("fuzz_decode.vcf.gz")


def test_header_only_is_error():
    st, dec = E.emu_decompress(bytes.fromhex(G.edge_cases()["header"]))
    assert st == E_FORMAT and dec == b""


@pytest.mark.parametrize("seed", [1, 2])
def test_valid_files_match_oracle(seed):
    for name, data in D.valid_files(seed):
        check(data, name)


@pytest.mark.parametrize("seed", [3, 4])
def test_mutated_files_match_oracle(seed):
    for name, data in D.mutated_files(seed):
        check(data, name)
