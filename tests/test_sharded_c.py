"""The multi-device engine (include/nghttp2_amd_hd.h nghttp2_amd_hd_sharded_*)
driven from C: tests/c/test_sharded.c links the library and, as its checker
only, the oracle (oracle/_build/libhuff_oracle.so).  CPU: it builds and
links.  GPU: 1, 2 and 3 shards of device 0 (worker threads, streams, device
contexts), host- and device-resident, bit-exact against the unsharded oracle
result, overflow without a byte past dst_cap."""
import os
import subprocess
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(REPO, "nghttp2_amd", "lib")
ORACLE = os.path.join(REPO, "oracle", "_build")


def build_c_test(outdir):
    from oracle import oracle as O
    O.lib()  # builds oracle/_build/libhuff_oracle.so when missing
    exe = os.path.join(outdir, "test_sharded")
    subprocess.run(["gcc", "-O1", "-Wall", "-D__HIP_PLATFORM_AMD__", "-I", os.path.join(REPO, "include"),
                    "-I", "/opt/rocm/include", os.path.join(REPO, "tests", "c", "test_sharded.c"),
                    "-L" + LIBDIR, "-lnghttp2_amd_hd", "-L" + ORACLE, "-lhuff_oracle",
                    "-L/opt/rocm/lib", "-lamdhip64",
                    "-Wl,-rpath," + LIBDIR, "-Wl,-rpath," + ORACLE, "-Wl,-rpath,/opt/rocm/lib",
                    "-o", exe], check=True)
    return exe


def test_c_sharded_program_links():
    with tempfile.TemporaryDirectory() as d:
        assert os.path.exists(build_c_test(d))


@pytest.mark.gpu
def test_c_sharded_program_runs(dev):
    with tempfile.TemporaryDirectory() as d:
        exe = build_c_test(d)
        r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        assert "sharded OK" in r.stdout
