"""CPU checks of the C-ABI boundary: the library loads, exports every symbol include/slatedb_amd.h
declares, its struct layouts match the header byte for byte, and host-only logic (sizing, argument
checks, the no-device error path) behaves.  No compute call runs here."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import pytest

from slatedb_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "slatedb_amd.h")


def header_functions():
    txt = open(HDR).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(sdb_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    from slatedb_amd import runtime
    return runtime.lib()


def test_exports_every_declared_symbol(lib):
    names = header_functions()
    assert len(names) >= 20
    out = subprocess.check_output(["nm", "-D", "--defined-only", os.path.join(ROOT, "slatedb_amd", "libslatedb_amd.so")]).decode()
    exported = set(re.findall(r" T (sdb_\w+)", out))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    assert set(names) == set(_abi.SIGNATURES), "ctypes signatures out of sync with the header"
    for n in names:
        getattr(lib, n)


STRUCTS = {
    "sdb_sst_view": _abi.SstView,
    "sdb_lookup_out": _abi.LookupOut,
    "sdb_footer_in": _abi.FooterIn,
    "sdb_kv_batch": _abi.KvBatch,
    "sdb_sst_params": _abi.SstParams,
    "sdb_sst_summary": _abi.SstSummary,
    "sdb_sst_out": _abi.SstOut,
    "sdb_decode_summary": _abi.DecodeSummary,
    "sdb_decoded_out": _abi.DecodedOut,
    "sdb_sst_host_result": _abi.SstHostResult,
    "sdb_decode_host_result": _abi.DecodeHostResult,
}


def test_struct_layouts_match_header():
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "%s"' % HDR, "int main(void){"]
    for cname, py in STRUCTS.items():
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for f, _ in py._fields_:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, f, cname, f))
    lines.append("return 0;}")
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "l.c"), os.path.join(d, "l")
        open(src, "w").write("\n".join(lines))
        subprocess.check_call(["gcc", "-std=c11", "-o", exe, src])
        out = dict(l.split() for l in subprocess.check_output([exe]).decode().splitlines())
    for cname, py in STRUCTS.items():
        assert int(out[cname]) == C.sizeof(py), cname
        for f, _ in py._fields_:
            assert int(out["%s.%s" % (cname, f)]) == getattr(py, f).offset, (cname, f)


def test_host_sizing_matches_oracle(lib):
    from oracle import oracle as O
    for n in (0, 1, 7, 100, 578524, 10_000_000, 429496730):
        for bpk in (1, 7, 10, 16):
            assert lib.sdb_bloom_filter_bytes(n, bpk) == O.filter_size_bytes(n, bpk), (n, bpk)
    for bpk in range(0, 40):
        assert lib.sdb_bloom_num_probes(bpk) == O.optimal_num_probes(bpk)
    assert lib.sdb_abi_version() == 2
    assert lib.sdb_status_name(3) == b"CHECKSUM_MISMATCH"


def test_bounds_and_argument_checks(lib):
    p = _abi.SstParams(4096, 2, 16, 10, 0)
    dc, bc, fc = C.c_uint64(), C.c_uint64(), C.c_uint64()
    assert lib.sdb_encode_bounds(578524, 578524 * 16, 578524 * 100, C.byref(p), C.byref(dc), C.byref(bc), C.byref(fc)) == 0
    assert dc.value >= 68455271 and bc.value >= 17016 and fc.value >= 723155
    bad = _abi.SstParams(4096, 3, 16, 10, 0)
    assert lib.sdb_encode_bounds(1, 1, 1, C.byref(bad), None, None, None) == _abi.SDB_INVALID_ARGUMENT
    bad = _abi.SstParams(4096, 2, 0, 10, 0)
    assert lib.sdb_encode_bounds(1, 1, 1, C.byref(bad), None, None, None) == _abi.SDB_INVALID_ARGUMENT
    assert lib.sdb_encode_workspace_bytes(1000, C.byref(p)) > 1000 * 32
    assert lib.sdb_decode_workspace_bytes(100) > 100 * 40


def test_no_device_fails_loudly(lib):
    """Without a GPU every compute entry point reports DEVICE_ERROR (no CPU fallback)."""
    if lib.sdb_device_count() > 0:
        pytest.skip("a HIP device is visible")
    p = _abi.SstParams(4096, 2, 16, 10, 0)
    b = _abi.KvBatch()
    sm = _abi.SstSummary()
    out = _abi.SstOut()
    out.summary = C.addressof(sm)
    assert lib.sdb_encode_sst(C.byref(b), C.byref(p), C.byref(out), None, 0, None) == _abi.SDB_DEVICE_ERROR
    assert lib.sdb_bloom_build(None, None, 0, 10, None, 0, None, 0, None) == _abi.SDB_DEVICE_ERROR
    assert not lib.sdb_encoder_create(0, C.byref(p))
    assert not lib.sdb_decoder_create(0)
    from slatedb_amd import runtime
    with pytest.raises(runtime.SdbError):
        runtime.Encoder()


# ------------------------------------------------------------------------------------------------
# INTEGRATION.md's Rust FFI structs must match the header (names, order, offsets, sizes)
# ------------------------------------------------------------------------------------------------
_RUST_PRIM = {"u8": (1, 1), "i8": (1, 1), "u16": (2, 2), "i16": (2, 2), "u32": (4, 4), "i32": (4, 4),
              "c_int": (4, 4), "u64": (8, 8), "i64": (8, 8), "f64": (8, 8), "usize": (8, 8)}


def rust_structs(md_path):
    txt = open(md_path).read()
    code = "\n".join(re.findall(r"```rust\n(.*?)```", txt, flags=re.S))
    out = {}
    for name, body in re.findall(r"#\[repr\(C\)\]\s*pub struct (\w+)\s*\{(.*?)\}", code, flags=re.S):
        body = re.sub(r"//[^\n]*", "", body)
        fields = re.findall(r"pub\s+(\w+)\s*:\s*([^,]+?)\s*(?:,|$)", body)
        if fields:
            out[name] = [(f, t.strip()) for f, t in fields]
    return out


def rust_layout(structs, name):
    """C layout (offsets, size, align) of a #[repr(C)] struct from its Rust field types."""
    off, align, offs = 0, 1, {}
    for f, t in structs[name]:
        if t.startswith("*"):
            sz = al = 8
        elif t in _RUST_PRIM:
            sz, al = _RUST_PRIM[t]
        else:
            _, sz, al = rust_layout(structs, t)
        off = (off + al - 1) // al * al
        offs[f] = off
        off += sz
        align = max(align, al)
    return offs, (off + align - 1) // align * align, align


def test_integration_rust_structs_match_header():
    structs = rust_structs(os.path.join(ROOT, "INTEGRATION.md"))
    want = ["sdb_kv_batch", "sdb_sst_params", "sdb_sst_summary", "sdb_sst_out", "sdb_sst_host_result",
            "sdb_footer_in", "sdb_decode_summary", "sdb_decoded_out", "sdb_decode_host_result", "sdb_sst_view",
            "sdb_lookup_out", "sdb_run", "sdb_retention", "sdb_merge_summary", "sdb_merged_out",
            "sdb_compacted_sst", "sdb_compaction_input"]
    missing = [w for w in want if w not in structs]
    assert not missing, missing
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "%s"' % HDR, "int main(void){"]
    for cname in structs:
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for f, _ in structs[cname]:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, f, cname, f))
    lines.append("return 0;}")
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "r.c"), os.path.join(d, "r")
        open(src, "w").write("\n".join(lines))
        subprocess.check_call(["gcc", "-std=c11", "-o", exe, src])
        got = dict(l.split() for l in subprocess.check_output([exe]).decode().splitlines())
    for cname in structs:
        offs, size, _ = rust_layout(structs, cname)
        assert int(got[cname]) == size, (cname, "size", size, got[cname])
        for f, off in offs.items():
            assert int(got["%s.%s" % (cname, f)]) == off, (cname, f)
    # every field of the header struct appears in the binding (no field silently missing)
    hdr = re.sub(r"/\*.*?\*/", "", open(HDR).read(), flags=re.S)
    for cname in want:
        m = re.search(r"typedef struct %s\s*\{(.*?)\}\s*%s;" % (cname, cname), hdr, flags=re.S)
        assert m, cname
        cfields = []
        for stmt in m.group(1).split(";"):
            parts = [x.strip() for x in stmt.split(",") if x.strip()]
            if parts:
                cfields += [re.findall(r"(\w+)\s*$", x)[0] for x in parts]
        assert [f for f, _ in structs[cname]] == cfields, (cname, [f for f, _ in structs[cname]], cfields)


def test_integration_declares_every_entry_point():
    """Every function of include/slatedb_amd.h (diagnostics aside) has a Rust declaration in INTEGRATION.md."""
    txt = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    code = "\n".join(re.findall(r"```rust\n(.*?)```", txt, flags=re.S))
    declared = set(re.findall(r"pub fn (sdb_\w+)\s*\(", code))
    want = {f for f in header_functions() if not f.startswith("sdb_diag_")}
    missing = sorted(want - declared)
    assert not missing, missing
