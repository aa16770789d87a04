"""The Rust binding (rust/fftconv_amd, written blind: no Rust toolchain in
this image) cannot drift from the C ABI: its extern declarations are generated
from include/fftconv.h, and every entry point the safe wrappers call is
declared with the header's arity."""
import os
import re
import subprocess
import sys

from conftest import ROOT

CRATE = os.path.join(ROOT, "rust", "fftconv_amd")


def test_ffi_rs_is_generated_from_the_header():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "gen_rust_ffi.py"), "--check"])
    assert r.returncode == 0, "rust/fftconv_amd/src/ffi.rs is stale: run scripts/gen_rust_ffi.py"


def test_wrappers_call_declared_functions_with_header_arity():
    ffi = open(os.path.join(CRATE, "src", "ffi.rs")).read()
    decl = {m.group(1): (m.group(2).count(":") if m.group(2).strip() else 0)
            for m in re.finditer(r"pub fn (fftconv_\w+)\(([^)]*)\)", ffi)}
    header = open(os.path.join(ROOT, "include", "fftconv.h")).read()
    for name in re.findall(r"\b(fftconv_\w+)\s*\(", header):
        assert name in decl, f"{name} missing from ffi.rs"
    lib = open(os.path.join(CRATE, "src", "lib.rs")).read()
    called = set(re.findall(r"ffi::(fftconv_\w+)\(", lib)) | set(re.findall(r"\b(fftconv_\w+)(?=[,)])", lib))
    for name in called:
        if name.startswith("fftconv_") and name not in ("fftconv_uniform", "fftconv_twostage", "fftconv_crossfade"):
            assert name in decl, f"lib.rs calls undeclared {name}"
    # every trait method of src/lib.rs:5-14 is implemented for the three types
    for ty in ("GpuFFTConvolver", "GpuTwoStageFFTConvolver", "GpuCrossfadeConvolver"):
        block = lib[lib.index(f"impl Convolution for {ty}"):]
        block = block[:block.index("\n}\n")]
        for m in ("fn init(", "fn update(", "fn reset(", "fn process("):
            assert m in block, f"{ty} lacks {m}"
