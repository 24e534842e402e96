"""The library's host path under AddressSanitizer + UBSan (host-side
sanitizer build).  Compiles the product source ``csrc/nf4_dequant_cpu.cpp`` with
the harness ``tests/asan/cpu_path_check.cpp`` and the C oracle (the checker),
runs every case with exactly-sized heap buffers and compares with the oracle
bit for bit.  Host code only: GPU sanitizers are not available on this pool."""
from __future__ import annotations

import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined", "-g"]


def _build(tmp_path):
    # the library's own host compiler (ROCm clang: _Float16 on x86, its compiler-rt
    # carries the ASan / UBSan runtimes); gcc only for the C oracle
    cxx = "/opt/rocm/llvm/bin/clang++" if os.path.exists("/opt/rocm/llvm/bin/clang++") else shutil.which("clang++")
    cc = shutil.which("gcc")
    if not cxx or not cc:
        pytest.skip("no host compiler")
    oracle_o = tmp_path / "oracle.o"
    exe = tmp_path / "cpu_path_check"
    # the oracle as plain C (its OpenMP pragmas ignored; the checker, not
    # instrumented: gcc's and clang's sanitizer runtimes do not mix), the product
    # source and the harness as instrumented C++
    cmds = [
        [cc, "-O1", "-std=c11", "-fno-fast-math", "-ffp-contract=off", "-g", "-c", "-o", str(oracle_o),
         os.path.join(REPO, "oracle", "nf4_oracle.c")],
        [cxx, "-O1", "-std=c++17", "-fno-fast-math", "-ffp-contract=off", "-pthread", *SAN, "-o", str(exe),
         os.path.join(REPO, "tests", "asan", "cpu_path_check.cpp"),
         os.path.join(REPO, "nf4_triton_dequantization_amd", "csrc", "nf4_dequant_cpu.cpp"), str(oracle_o)],
    ]
    for c in cmds:
        r = subprocess.run(c, capture_output=True, text=True)
        if r.returncode != 0:
            if "asan" in r.stderr.lower() or "sanitizer" in r.stderr.lower():
                pytest.skip(f"sanitizer runtime unavailable: {r.stderr[-300:]}")
            raise AssertionError(f"build failed: {' '.join(c)}\n{r.stderr[-2000:]}")
    return exe


def test_host_path_under_address_and_ub_sanitizers(tmp_path):
    exe = _build(tmp_path)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None) if "libasan" in env.get("LD_PRELOAD", "") else None
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, f"rc={r.returncode}\nstdout={r.stdout[-2000:]}\nstderr={r.stderr[-4000:]}"
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    assert '"failures": 0' in r.stdout, r.stdout
