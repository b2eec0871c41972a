"""The C-ABI library loads on a CPU-only host, exports every symbol the headers
declare (include/honu_codec.h: the drop-in boundary; include/honu_bench.h:
the generator, digests, verifier and probe the bench and tests use), and its
struct layouts match the host-side numpy views."""
import os
import re
import subprocess

import numpy as np
import pytest

from honu_amd import _lib
from honu_amd.metadata import ACL_DTYPE, INFO_DTYPE, META_DTYPE
from honu_amd.system import COLLECTION_DTYPE, INDEX_DTYPE

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "honu_codec.h")
BENCH_HEADER = os.path.join(ROOT, "include", "honu_bench.h")


def header_functions(paths=(HEADER, BENCH_HEADER)):
    names = set()
    for path in paths:
        src = re.sub(r"/\*.*?\*/", "", open(path).read(), flags=re.S)
        names |= set(re.findall(r"\b(honu_[a-z0-9_]+)\s*\(", src))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    names = header_functions()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(_lib.EXPORTS)


def test_product_header_is_the_binding():
    """The product header holds what INTEGRATION.md binds; the measurement
    entry points live in honu_bench.h only."""
    product = set(header_functions((HEADER,)))
    bench_only = set(header_functions((BENCH_HEADER,))) - product
    assert {"honu_gen_meta", "honu_digest_records", "honu_verify_decoded", "honu_hbm_probe"} <= bench_only
    assert not product & {"honu_gen_totals", "honu_gen_payload", "honu_digest_host"}


STRUCTS = ((META_DTYPE, "honu_meta"), (ACL_DTYPE, "honu_acl"), (INFO_DTYPE, "honu_record_info"),
           (COLLECTION_DTYPE, "honu_collection"), (INDEX_DTYPE, "honu_index"))


def test_abi_self_description():
    lib = _lib.load()
    assert lib.honu_abi_version() == 6
    assert lib.honu_sizeof_meta() == META_DTYPE.itemsize == 352
    assert lib.honu_sizeof_acl() == ACL_DTYPE.itemsize == 20
    assert lib.honu_sizeof_record_info() == INFO_DTYPE.itemsize == 32
    assert lib.honu_sizeof_collection() == COLLECTION_DTYPE.itemsize == 368
    assert lib.honu_sizeof_index() == INDEX_DTYPE.itemsize == 112
    assert lib.honu_status_string(2).decode().startswith("object is malformed")


def test_struct_offsets_match_numpy(tmp_path):
    """Compile offsetof() of every field with the system C compiler."""
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(){"]
    for dt, ct in STRUCTS:
        for name in dt.names:
            lines.append(f'printf("{ct}.{name} %zu\\n", offsetof({ct}, {name}));')
    lines.append("return 0;}")
    c = tmp_path / "off.c"
    c.write_text("\n".join(lines))
    exe = tmp_path / "off"
    subprocess.run(["gcc", "-std=c11", "-o", str(exe), str(c)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    got = dict(line.rsplit(" ", 1) for line in out.strip().splitlines())
    for dt, ct in STRUCTS:
        for name in dt.names:
            assert int(got[f"{ct}.{name}"]) == dt.fields[name][1], (ct, name)


def test_product_library_reads_no_environment():
    """The product library behaves the same whatever the caller's process
    environment holds: it imports no getenv at all, so
    HONU_ACL_INPLACE=0 and the like cannot change its outputs; only the A/B
    build (make ab) reads HONU_* variables. (tests/test_gpu_parity.py
    test_environment_is_ignored checks the same on the GPU.)"""
    if _lib.LIB_PATH != os.path.join(ROOT, "honu_amd", "libhonu_codec.so"):
        pytest.skip("HONU_LIB_PATH points at another build")
    out = subprocess.run(["nm", "-D", "--undefined-only", _lib.LIB_PATH], check=True,
                         capture_output=True, text=True).stdout
    imported = {ln.split()[-1].split("@")[0] for ln in out.splitlines() if ln.strip()}
    assert not imported & {"getenv", "secure_getenv", "__secure_getenv"}, imported & {"getenv"}
    ab = os.path.join(ROOT, "honu_amd", "libhonu_codec_ab.so")
    if os.path.exists(ab):  # the measurement build does read them
        out = subprocess.run(["nm", "-D", "--undefined-only", ab], check=True, capture_output=True,
                             text=True).stdout
        assert "getenv" in out


def test_no_gpu_fails_loudly():
    """Without a gfx950 device the context cannot be created (no CPU fallback)."""
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    lib = _lib.load()
    err = _lib.I32(0)
    ctx = lib.honu_ctx_create(0, 16, _lib.C.byref(err))
    assert not ctx and err.value == -4


def test_host_generator_is_deterministic():
    lib = _lib.load()
    tot = np.zeros(4, np.uint64)
    lib.honu_gen_totals(7, 4, 100, 300, tot.ctypes.data)
    n = 300
    meta = np.zeros(n, META_DTYPE)
    var = np.zeros(int(tot[0]), np.uint8)
    acl = np.zeros(max(int(tot[1]), 1), ACL_DTYPE)
    reg = np.zeros(max(int(tot[2]), 1), np.uint32)
    off = np.zeros(n + 1, np.uint64)
    lib.honu_gen_meta(7, 4, 100, n, meta.ctypes.data, var.ctypes.data, acl.ctypes.data,
                      reg.ctypes.data, off.ctypes.data)
    assert int(off[n]) == int(tot[3])
    # records are a function of (seed, index): the same records from a shifted window
    meta2 = np.zeros(n - 50, META_DTYPE)
    tot2 = np.zeros(4, np.uint64)
    lib.honu_gen_totals(7, 4, 150, n - 50, tot2.ctypes.data)
    var2 = np.zeros(int(tot2[0]), np.uint8)
    acl2 = np.zeros(max(int(tot2[1]), 1), ACL_DTYPE)
    reg2 = np.zeros(max(int(tot2[2]), 1), np.uint32)
    off2 = np.zeros(n - 49, np.uint64)
    lib.honu_gen_meta(7, 4, 150, n - 50, meta2.ctypes.data, var2.ctypes.data, acl2.ctypes.data,
                      reg2.ctypes.data, off2.ctypes.data)
    for f in ("pid", "vid", "region", "created", "acl_count", "regions_count", "present", "owner"):
        assert np.array_equal(meta[50:][f], meta2[f]), f
    assert np.array_equal(np.diff(off[50:]), np.diff(off2))
