"""Host code under sanitizers (the reference's tests run with
-race, test.sh:57-69).  scripts/build_sanitizers.sh builds the library with
qe_pack.cpp under ASan+UBSan and under TSan, and the C oracle under
ASan+UBSan; the packing tests (tests/test_packing.py, the multi-threaded
tests/test_pack_threads.py) and the oracle's golden tests
(tests/test_oracle_golden.py, tests/test_progress_oracle.py) then run
against them in a child interpreter with gcc's runtimes preloaded (Python
itself is not instrumented).  Any report fails the child (halt_on_error)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "etcd_amd", "build_san")


def _rt(name):
    return subprocess.check_output(["gcc", f"-print-file-name={name}"], text=True).strip()


@pytest.fixture(scope="module")
def built():
    subprocess.check_call(["bash", os.path.join(ROOT, "scripts", "build_sanitizers.sh")],
                          stdout=subprocess.DEVNULL)
    return SAN


def _run(env_extra, tests):
    env = dict(os.environ)
    env.update(env_extra)
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                        "-m", "not gpu"] + tests, cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert "WARNING: ThreadSanitizer" not in out, out[-4000:]
    return out


def test_packer_under_asan_ubsan(built):
    _run({"QE_LIB": os.path.join(built, "libetcd_quorum_asan.so"),
          "LD_PRELOAD": f"{_rt('libasan.so')} {_rt('libubsan.so')}",
          "ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1",
          "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"},
         ["tests/test_packing.py", "tests/test_pack_threads.py"])


def test_packer_threads_under_tsan(built):
    _run({"QE_LIB": os.path.join(built, "libetcd_quorum_tsan.so"),
          "LD_PRELOAD": _rt("libtsan.so"),
          "TSAN_OPTIONS": "halt_on_error=1:report_signal_unsafe=0"},
         ["tests/test_packing.py", "tests/test_pack_threads.py"])


def test_oracle_under_asan_ubsan(built):
    _run({"QE_ORC_LIB": os.path.join(built, "liborc_asan.so"),
          "LD_PRELOAD": f"{_rt('libasan.so')} {_rt('libubsan.so')}",
          "ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1",
          "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"},
         ["tests/test_oracle_golden.py", "tests/test_progress_oracle.py",
          "tests/test_propose_oracle.py", "tests/test_trace_replay.py"])
