"""Host sanitizers over the native runtime (csrc/runtime): the block manager and step builders are
compiled with AddressSanitizer + UndefinedBehaviorSanitizer into a standalone self-test
(csrc/runtime/tests/runtime_selftest.cpp: randomized model check of every block-manager operation
against a shadow reference count, step builders writing into exactly-sized heap buffers) and run on
the CPU. GPU sanitizers are not available on the MI355X pool; this is the memory-safety and
UB check of the runtime's host code (SURVEY §5 "race detection / sanitizers")."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RT = os.path.join(ROOT, "csrc", "runtime")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_runtime_selftest_asan_ubsan(tmp_path):
    exe = tmp_path / "runtime_selftest"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=undefined", "-I", RT, os.path.join(RT, "tests", "runtime_selftest.cpp"),
                    "-o", str(exe)], check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([str(exe), "20000", "7"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "runtime selftest ok" in r.stdout and "LRU evictions" in r.stdout
