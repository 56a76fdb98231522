"""The C-ABI boundary without a GPU: wire-struct layout, exported symbols, the header compiling
as C and C++, and the host-side validation paths of KernelWrapper (which return before any HIP
call). Compute entry points are exercised by tests/test_gpu_parity.py on the MI355X."""
import ctypes as C
import re
import struct
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "mh_kernel.h"


def test_struct_layout_matches_reference(mh):
    for cls, (size, offsets) in mh.STRUCT_LAYOUT.items():
        assert C.sizeof(cls) == size, cls.__name__
        for field, off in offsets.items():
            assert getattr(cls, field).offset == off, (cls.__name__, field)


def test_library_exports_every_declared_symbol(mh, hiplib):
    declared = set(re.findall(r"MH_API\s+[\w\s\*]+?\b(\w+)\s*\(", HEADER.read_text()))
    assert declared == set(mh.EXPORTS)
    out = subprocess.run(["nm", "-D", "--defined-only", str(mh.LIB_PATH)], check=True,
                         capture_output=True, text=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    assert declared <= exported, declared - exported
    for name in declared:
        assert hasattr(hiplib, name)


def test_library_is_gfx950_code(mh, tmp_path):
    """The offload bundle carries a gfx950 code object (extracted in a scratch dir)."""
    lib = tmp_path / mh.LIB_PATH.name
    lib.write_bytes(mh.LIB_PATH.read_bytes())
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib)],
                         capture_output=True, text=True, cwd=tmp_path)
    assert "gfx950" in (out.stdout + out.stderr) or b"gfx950" in lib.read_bytes()


def _device_functions(lib_path, tmp_path):
    """Names of the FUNC symbols of every gfx950 code object in the library's offload bundles
    (one bundle per HIP translation unit, concatenated in .hip_fatbin)."""
    fatbin = tmp_path / "fatbin.bin"
    subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objcopy", f"--dump-section=.hip_fatbin={fatbin}",
                    str(lib_path), str(tmp_path / "stripped.so")], check=True)
    data = fatbin.read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    names, objects = set(), 0
    at = data.find(magic)
    while at >= 0:
        count = struct.unpack_from("<Q", data, at + 24)[0]
        p = at + 32
        for _ in range(count):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" not in triple:
                continue
            co = tmp_path / f"co{objects}.o"
            co.write_bytes(data[at + off:at + off + size])
            objects += 1
            out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-s", "--wide", str(co)],
                                 check=True, capture_output=True, text=True).stdout
            for ln in out.splitlines():
                f = ln.split()
                if len(f) >= 8 and f[3] == "FUNC":
                    names.add(f[7])
        at = data.find(magic, at + 1)
    return names, objects


def test_step_kernels_make_no_calls(mh, tmp_path):
    """Every device function that takes references to a kernel's private objects (eval_costs,
    propose, the incremental kernel's helpers) is inlined: an out-of-line call of eval_costs
    faulted on MI355X (DESIGN.md "The counting-build fault"). Only value-only helpers may stay
    out of line: the Box-Muller transforms, the rare-path transcendentals (mh_common.h) and the
    speculative kernel's Philox words past its window."""
    names, objects = _device_functions(mh.LIB_PATH, tmp_path)
    assert objects == 5  # mh_chain, mh_chain_xw, mh_chain_best, mh_delta, mh_spec
    kernels = {n for n in names if "_kernel" in n}
    assert any("mh_kernelILi64ELi1ELi1E" in n for n in kernels)
    helpers = names - kernels
    allowed = {"_ZN2mhL10box_mullerEjj", "_ZN2mhL17curand_box_mullerEjj", "_ZN2mhL9atan2_oolEdd",
               "_ZN2mhL11cos_f32_oolEf", "_ZN2mhL7exp_oolEd",
               "_ZN2mh12_GLOBAL__N_110philox_farEmmm"}  # (mh_spec.hip: redraws past the window)
    assert helpers <= allowed, sorted(helpers - allowed)


_BYTE_TYPES = {"char", "unsigned char", "signed char", "uint8_t", "std::byte", "void"}
# the LDS carve-up: `lds` is the extern __shared__ unsigned char array and `base` a chain's byte
# pointer into it; a typed array placed there is only ever accessed through its own type
_BYTE_POINTERS = {"lds", "base", "s->d_meta"}


def test_no_type_punning():
    """No memory is read or written through a pointer cast between unrelated object types
    (strict aliasing; the class of undefined behaviour DESIGN.md "The counting-build fault" blames
    for round 3's wrong code out of line). Allowed: casts to byte pointers, and casts from the LDS
    byte pointers that place a typed array. Vector views of other types go through load16()
    (mh_common.h), a value copy."""
    csrc = ROOT / "metropolis-hastings-gpgpu_amd" / "csrc"
    text = {f.name: f.read_text() for f in sorted(csrc.iterdir())
            if f.suffix in (".hip", ".h", ".cpp")}
    text["mh_kernel.h"] = HEADER.read_text()
    cast = re.compile(r"reinterpret_cast<\s*(?:const\s+)?([\w:\s]+?)\s*(?:const\s*)?\*\s*>\s*\(\s*"
                      r"(&?[\w\->\.]+)")
    bad = []
    for name, src in text.items():
        for m in cast.finditer(src):
            target, operand = m.group(1).strip(), m.group(2)
            if target in _BYTE_TYPES or operand in _BYTE_POINTERS:
                continue
            bad.append(f"{name}:{src.count(chr(10), 0, m.start()) + 1}: {m.group(0)}")
        # C-style pointer casts and unions are not used for punning either
        for m in re.finditer(r"\(\s*(?:const\s+)?(?:float|double|u?int\d*_t|int|unsigned|u?int[24]|"
                             r"float[24]|double2)\s*\*\s*\)\s*&", src):
            bad.append(f"{name}:{src.count(chr(10), 0, m.start()) + 1}: {m.group(0)}")
        for m in re.finditer(r"\bunion\b", src):
            bad.append(f"{name}:{src.count(chr(10), 0, m.start()) + 1}: union")
    assert not bad, "type punning:\n" + "\n".join(bad)
    # the byte pointers really are byte pointers
    assert "extern __shared__ __attribute__((aligned(16))) unsigned char lds[];" in text["mh_chain.hip"]
    assert "unsigned char* base = lds" in text["mh_chain.hip"]
    assert "unsigned char* base = lds" in text["mh_delta.hip"]


@pytest.mark.parametrize("lang,compiler", [("c", "gcc"), ("c++", "g++")])
def test_header_compiles_and_links(mh, tmp_path, lang, compiler):
    src = tmp_path / ("t.c" if lang == "c" else "t.cpp")
    src.write_text("""
#include "mh_kernel.h"
#include <stdio.h>
int main(void) {
    result* (*kw)(relationshipStruct*, relationshipAngleStruct*, positionAndRotation*,
                  rectangle*, rectangle*, vertex*, vertex*, Surface*, gpuConfig*) = KernelWrapper;
    printf("%d %d %p\\n", (int)sizeof(result), (int)sizeof(Surface), (void*)kw);
    KernelFreeResult(0);
    return 0;
}
""")
    exe = tmp_path / "t"
    subprocess.run([compiler, "-std=c11" if lang == "c" else "-std=c++17", "-Wall", "-Werror",
                    "-I", str(ROOT / "include"), str(src), "-o", str(exe),
                    str(mh.LIB_PATH), f"-Wl,-rpath,{mh.LIB_PATH.parent}"], check=True)


def _call(hiplib, mh, room, chains=4, iters=10):
    g = mh.abi.gpuConfig(chains, 0, 64, 0, 0, iters)
    return hiplib.KernelWrapperSeeded(*room.args(), C.byref(g), C.c_uint64(1))


@pytest.mark.parametrize("breaker,needle", [
    (lambda r: setattr(r.srf, "nObjs", 0), "nObjs"),
    (lambda r: setattr(r.srf, "nClearances", 40), "nClearances"),
    (lambda r: setattr(r.rss[0], "TargetIndex", 99), "relationship"),
    (lambda r: setattr(r.clearances[1], "SourceIndex", -1), "SourceIndex"),
    (lambda r: setattr(r.offlimits[3], "point1Index", 500), "point1Index"),
])
def test_invalid_rooms_return_null_with_message(mh, hiplib, breaker, needle):
    room = mh.main_fixture()
    breaker(room)
    assert not _call(hiplib, mh, room)
    assert needle in mh.last_error(hiplib)


def test_all_frozen_is_an_error_not_a_hang(mh, hiplib):
    room = mh.synthetic_room(8, freeze_every=1)
    assert not _call(hiplib, mh, room)
    assert "frozen" in mh.last_error(hiplib)


def test_bad_gpu_config(mh, hiplib):
    room = mh.main_fixture()
    assert not _call(hiplib, mh, room, chains=0)
    assert "gridxDim" in mh.last_error(hiplib)
    assert not _call(hiplib, mh, room, iters=-1)
    assert "iterations" in mh.last_error(hiplib)


def test_null_arguments(mh, hiplib):
    room = mh.main_fixture()
    g = mh.abi.gpuConfig(1, 0, 64, 0, 0, 1)
    args = list(room.args())
    args[7] = None  # srf
    assert not hiplib.KernelWrapper(*args, C.byref(g))
    assert "srf" in mh.last_error(hiplib)
    assert not hiplib.KernelWrapper(*room.args(), None)
    hiplib.KernelFreeResult(None)


def test_debug_math_buffer_sized_from_probe(mh, orc):
    """mh_debug_math writes mh_probe_width(fn) doubles per argument: the wrapper sizes its buffer
    from the probe id (the oracle's table agrees) and rejects a width that disagrees before any
    call."""
    for fn in range(mh.MH_PROBE_COUNT):
        assert mh.probe_width(fn) == orc.probe_width(fn), fn
    with pytest.raises(ValueError):
        mh.debug_math(1, 0, 4, 1)  # a sincos probe writes 2
    with pytest.raises(ValueError):
        mh.debug_math(mh.MH_PROBE_COUNT, 0, 4)


def test_cross_lane_lds_hand_offs_are_named():
    """Every cross-lane LDS hand-off of the kernels goes through mh_common.h's views (VERDICT round
    5, item 6): no bare wave_sync() outside mh_common.h; the full-evaluation and incremental
    kernels' chain arrays are Published members (a plain assignment to one does not compile, a
    write goes through stage()), and each of their phases ends in a hand_off() naming arrays."""
    csrc = ROOT / "metropolis-hastings-gpgpu_amd" / "csrc"
    for f in sorted(csrc.iterdir()):
        if f.suffix in (".hip", ".cpp") or (f.suffix == ".h" and f.name != "mh_common.h"):
            src = f.read_text()
            assert not re.search(r"\bwave_sync\s*\(\s*\)", src), f"bare wave_sync() in {f.name}"
    chain = (csrc / "mh_chain.hip").read_text()
    delta = (csrc / "mh_delta.hip").read_text()
    for src, struct, arrays in ((chain, "ChainPtrs", ("P", "PX", "LCL", "CLA", "NZ", "aux")),
                                (delta, "DeltaPtrs", ("X", "BOX", "CPH", "LCL", "SAM", "aux"))):
        body = src[src.index(f"struct {struct} {{"):]
        body = body[:body.index("};")]
        for a in arrays:
            assert re.search(rf"Published<[\w]+> [^;]*\b{a}\b", body), f"{struct}.{a} not Published"
        assert len(re.findall(r"\bhand_off\(ch\.", src)) >= 10
