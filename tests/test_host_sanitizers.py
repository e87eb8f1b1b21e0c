"""The library's pure C++ host code (DIMACS loader, `solve` preprocessing, experiment knobs) under
AddressSanitizer + UndefinedBehaviorSanitizer (host-side only; GPU sanitizers are not available on the
pool): tests/sanitize/host_fuzz.cpp runs the reference's three fixture files, mutated copies of them,
and random DIMACS texts (empty clauses, duplicate literals, huge variable names, missing headers) and
their mutations through parse -> export -> normalize -> evaluate -> memories -> preprocess -> trace ->
tri-state evaluation.  Any out-of-bounds access, use after free, leak or undefined behaviour aborts the run."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "odesat_amd", "csrc")


def test_host_code_under_asan_and_ubsan(tmp_path):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    exe = tmp_path / "host_fuzz"
    build = subprocess.run([cxx, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                            "-fno-omit-frame-pointer", "-o", str(exe), os.path.join(ROOT, "tests", "sanitize", "host_fuzz.cpp"),
                            os.path.join(CSRC, "cnf.cpp"), os.path.join(CSRC, "preprocess.cpp"),
                            os.path.join(CSRC, "experiment.cpp")], capture_output=True, text=True)
    assert build.returncode == 0, build.stderr
    golden = [os.path.join(ROOT, "tests", "golden", f) for f in ("easy.cnf", "hard.cnf", "small.cnf")]
    r = subprocess.run([str(exe), "120", "7", *golden], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed checks" in r.stdout
