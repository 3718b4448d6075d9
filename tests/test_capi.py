"""C-ABI library: builds, loads, exports every symbol include/vcfc.h declares,
and fails loudly (no CPU fallback) when no GPU is visible."""
import ctypes
import os
import re
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "build", "libvcfc.so")


def declared_symbols():
    src = open(os.path.join(REPO, "include", "vcfc.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vcfc_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "vcf-compression_amd")], check=True)
    return ctypes.CDLL(LIB)


def test_exports_every_declared_symbol(lib):
    syms = declared_symbols()
    assert len(syms) >= 15
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_lists_all_exports():
    import sys
    sys.path.insert(0, os.path.join(REPO, "vcf-compression_amd"))
    import vcfc
    assert sorted(vcfc.EXPORTS) == declared_symbols()


def test_code_object_is_gfx950(lib):
    blob = open(LIB, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in blob


def test_strerror_and_bounds(lib):
    lib.vcfc_strerror.restype = ctypes.c_char_p
    assert b"8 terms" in lib.vcfc_strerror(1)
    lib.vcfc_encode_bound.restype = ctypes.c_uint64
    lib.vcfc_encode_bound.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
    assert lib.vcfc_encode_bound(10, 1000) >= 1000 * 3 // 2


def test_workspace_staging_primary_per_batch(lib):
    """The encode workspace holds prim_bytes of staging per row: 2 KiB for
    batches whose mean line is >= 4 KiB, else 1 KiB (vcfc_prim_bytes,
    vcfc_device.h); the rest scales with the line bytes."""
    lib.vcfc_encode_workspace_size.restype = ctypes.c_uint64
    lib.vcfc_encode_workspace_size.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
    ws = lib.vcfc_encode_workspace_size
    n = 100_000
    # one more byte of lines changes the line-dependent parts by a few bytes;
    # crossing the 4 KiB mean adds the second KiB of staging per row
    below, above = ws(n, n * 4096 - 1), ws(n, n * 4096)
    assert above - below >= 1024 * n
    assert above - below < 1024 * n + 4096
    # short rows keep 1 KiB per row: the workspace of 100-sample rows
    # (~420 B) stays within a few times their bytes
    assert ws(n, n * 420) < 6 * n * 420
    assert ws(0, 0) >= 0


def test_no_gpu_fails_loudly(lib):
    import torch  # noqa: F401  (device count only; does not initialise HIP)
    if torch.cuda.device_count() > 0:
        pytest.skip("GPU present")
    h = ctypes.c_void_p()
    lib.vcfc_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    assert lib.vcfc_ctx_create(0, ctypes.byref(h)) == 6  # VCFC_E_HIP


def test_links_the_real_hip_runtime_with_no_undefined_symbols(lib):
    """The library is linked against ROCm's libamdhip64 with -z defs (every
    symbol resolved at build time) and records it by soname, so a PyTorch
    process maps ONE HIP runtime (torch's copy has the same soname)."""
    d = subprocess.run(["/opt/rocm/llvm/bin/llvm-readelf", "-d", LIB], capture_output=True, text=True).stdout
    assert "[libamdhip64.so.7]" in d
    r = subprocess.run(["ldd", "-r", LIB], capture_output=True, text=True)
    assert "undefined symbol" not in r.stdout + r.stderr
    code = ("import sys; sys.path.insert(0, %r); import torch, vcfc; vcfc.lib(); "
            "print(sorted({l.split()[-1] for l in open('/proc/self/maps') if 'libamdhip64' in l}))"
            % os.path.join(REPO, "vcf-compression_amd"))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300).stdout
    assert out.count("libamdhip64") == 1, out


DIAG_SWITCHES = ["VCFC_DIAG_NOSTORE", "VCFC_DIAG_NOSTEP", "VCFC_DIAG_CLEAN_SKIP", "VCFC_VAR_SIZE_ONLY",
                 "VCFC_DIAG_DEC_NOSCAN", "VCFC_DIAG_NOESCEMIT",
                 "VCFC_DIAG_NODIRECT", "VCFC_DIAG_HOP_TWICE"]


@pytest.mark.parametrize("sw", DIAG_SWITCHES)
def test_diag_switches_refused(sw, tmp_path):
    """the kernels' wrong-output diagnostic switches can
    never reach libvcfc.so.  `make` refuses them without VCFC_DIAG_BUILD and
    refuses any diagnostic build into build/; the kernel sources refuse them
    at preprocessing (vcfc_device.h #error) without VCFC_DIAG_BUILD."""
    mk = os.path.join(REPO, "vcf-compression_amd")
    r = subprocess.run(["make", "-n", "-C", mk, "EXTRA=-D%s" % sw], capture_output=True, text=True)
    assert r.returncode != 0 and "wrong output" in r.stderr
    r = subprocess.run(["make", "-n", "-C", mk, "EXTRA=-D%s -DVCFC_DIAG_BUILD" % sw], capture_output=True, text=True)
    assert r.returncode != 0 and "may not replace the product library" in r.stderr
    src = "vcfc_decode.hip" if "DEC" in sw else "vcfc_encode.hip"
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-std=c++17", "-I", os.path.join(mk, "csrc"),
           "-I", os.path.join(REPO, "include"), "-D" + sw, "-E", os.path.join(mk, "csrc", src), "-o", os.devnull]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "diagnostic builds only" in r.stderr
    r = subprocess.run(cmd[:-4] + ["-DVCFC_DIAG_BUILD"] + cmd[-4:], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-400:]
