"""The host layers under AddressSanitizer + UndefinedBehaviorSanitizer
(the reference's CI does the same,
.github/workflows/build.yml:316-317).

`make -C nghttp2_amd asan` (run by __graft_entry__.build) instruments the
host code of the library -- the batched inflate front-end (hd_inflate.cpp,
which parses untrusted wire), the deflater (hd_deflate.cpp), the C ABI --
and links the hpack-test-case drivers (json_lite.h) and the harness
tests/c/host_sanitize.cpp with the sanitizer runtimes.  On the CPU they run:

- the reference's inflate cases, a randomized malformed-block fuzz over
  several inflaters and small output caps, static-table deflates inflated
  back, and mutated JSON documents (host_sanitize);
- the drivers' CPU tests (tests/test_drivers.py, not gpu) on the sanitized
  drivers.
Any sanitizer report fails the run (-fno-sanitize-recover, nonzero exit)."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN_BIN = os.path.join(REPO, "nghttp2_amd", "bin", "asan")
ENV = dict(os.environ, ASAN_OPTIONS="abort_on_error=0:halt_on_error=1:detect_leaks=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _need(tool):
    path = os.path.join(ASAN_BIN, tool)
    if not os.path.exists(path):
        pytest.fail("%s missing: build() (make -C nghttp2_amd asan) first" % path)
    return path


def _no_report(p):
    err = p.stderr.decode(errors="replace")
    assert "AddressSanitizer" not in err and "runtime error:" not in err and \
        "LeakSanitizer" not in err, err[-4000:]


@pytest.mark.parametrize("seed", [1, 2])
def test_host_layers_fuzz_under_asan(seed):
    p = subprocess.run([_need("host_sanitize"), os.path.join(REPO, "tests", "golden", "ref_hd_tests.json"),
                        "3000", str(seed)], capture_output=True, timeout=600, env=ENV)
    _no_report(p)
    assert p.returncode == 0, p.stderr.decode(errors="replace")[-4000:]
    out = p.stdout.decode()
    assert "host_sanitize: ok" in out
    assert "reference inflate cases: 7" in out


def test_drivers_under_asan():
    _need("deflatehd")
    _need("inflatehd")
    env = dict(ENV, NGHTTP2_AMD_BIN=ASAN_BIN)
    p = subprocess.run([sys.executable, "-m", "pytest", "-q", "-m", "not gpu", "-p", "no:cacheprovider",
                        os.path.join(REPO, "tests", "test_drivers.py")],
                       capture_output=True, timeout=600, env=env, cwd=REPO)
    assert p.returncode == 0, (p.stdout.decode()[-3000:], p.stderr.decode()[-3000:])
    assert " passed" in p.stdout.decode()
