"""The inflate front-end's three pinned-pool modes (NGHTTP2_AMD_INFLATE_ZC,
read once per process by nghttp2_amd/csrc/hd_inflate.cpp): 0 explicit H2D and
D2H copies, 1 the kernel reads and writes the mapped pools, 2 (default) it
reads the mapped input pools and its output is copied back.  Each mode runs
in a fresh child process with the variable set before any GPU call: RFC 7541
C.4 / C.6 (per block and batched), the random connections with corruptions,
and the reference's fuzz-corpus connections, all against the oracle."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
sys.path.insert(0, %r)
from tests import test_inflate as T
from tests import test_fuzz_corpus as F
for ex in T.EXAMPLES:
    if ex["huffman"]:
        T._check_example(ex, per_block=True)
        T._check_example(ex, per_block=False)
T.test_inflate_random_connections_vs_oracle()
F.test_fuzz_corpus_one_batch_vs_oracle()
print("ZC-OK")
""" % REPO


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["0", "1", "2"])
def test_inflate_pool_modes_vs_oracle(mode):
    env = dict(os.environ, NGHTTP2_AMD_INFLATE_ZC=mode)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, cwd=REPO,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "ZC-OK" in r.stdout, (mode, r.stdout[-2000:], r.stderr[-2000:])
