"""hpack-test-case drivers (nghttp2_amd/bin/deflatehd, inflatehd; SURVEY.md
8(f) row 3, BASELINE config 1) over the batched C ABI.

The reference tools (src/deflatehd.cc, src/inflatehd.cc) cannot be built
here (C++23 <print>, jansson), so their behaviour is pinned through the
library: the config-1 set's wire must equal the restated deflater's
(tests/golden/config1_wire.json, made by tests/golden/make_config1.py; the
restatement reproduces nghttp2's RFC 7541 C.4 output), and inflatehd must
give back every header.  Inputs whose fields all hit the static table make
no GPU call and run on the CPU; the rest are gpu tests."""
import json
import os
import subprocess

import pytest

from oracle import hpack_oracle as HO

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# NGHTTP2_AMD_BIN: another build of the drivers (tests/test_sanitize.py: the ASan one)
BIN = os.environ.get("NGHTTP2_AMD_BIN") or os.path.join(REPO, "nghttp2_amd", "bin")
GOLD = os.path.join(REPO, "tests", "golden")


def run(tool, args=(), stdin=b"", check=True):
    p = subprocess.run([os.path.join(BIN, tool), *args], input=stdin, capture_output=True,
                       timeout=120)
    if check and p.returncode != 0:
        raise AssertionError("%s failed (%d): %s" % (tool, p.returncode, p.stderr.decode()))
    return p


def headers_of(case):
    return [(k, v) for pair in case["headers"] for k, v in pair.items()]


STATIC_ONLY = {"context": "request", "cases": [
    {"headers": [{":method": "GET"}, {":scheme": "http"}, {":path": "/"}]},
    {"headers": []},
    {"headers": [{":status": "200"}, {"accept-encoding": "gzip, deflate"}]}]}

# the layout jansson's json_dumpf(JSON_INDENT(2) | JSON_PRESERVE_ORDER) gives
# the reference tool for the first case (src/deflatehd.cc:80-117)
FIRST_CASE_TEXT = """{
  "cases":
  [
{
  "seq": 0,
  "input_length": 27,
  "output_length": 3,
  "percentage_of_original_size": 11.111111111111111,
  "wire": "828684",
  "headers": [
    {
      ":method": "GET"
    },
    {
      ":scheme": "http"
    },
    {
      ":path": "/"
    }
  ],
  "header_table_size": 4096
}
,
"""


def test_deflatehd_format_cpu():
    p = run("deflatehd", stdin=json.dumps(STATIC_ONLY).encode())
    out = p.stdout.decode()
    assert out.startswith(FIRST_CASE_TEXT)
    assert out.endswith("}\n  ]\n}\n")
    doc = json.loads(out)
    assert [c["wire"] for c in doc["cases"]] == ["828684", "", "88" + "90"]
    assert doc["cases"][1]["percentage_of_original_size"] == 0.0
    assert "header_table_size" not in doc["cases"][1]
    assert p.stderr.decode().startswith("Overall: input=65 output=5 ratio=0.08")


def test_inflatehd_roundtrip_cpu():
    d = run("deflatehd", ["-d"], stdin=json.dumps(STATIC_ONLY).encode()).stdout
    dd = json.loads(d)
    assert all(c["header_table"] == {"entries": [], "size": 0, "max_size": 4096} for c in dd["cases"])
    i = json.loads(run("inflatehd", stdin=d).stdout)
    for a, b in zip(STATIC_ONLY["cases"], i["cases"]):
        assert headers_of(a) == headers_of(b)
        assert "header_table_size" not in b  # 4096 -> 4096: no change


def test_table_size_options_cpu():
    # -s 256: the first block opens with the size update (RFC 7541 6.3)
    d = json.loads(run("deflatehd", ["-s", "256"], stdin=json.dumps(STATIC_ONLY).encode()).stdout)
    assert d["cases"][0]["wire"] == "3fe101828684"
    assert d["cases"][0]["header_table_size"] == 256
    i = json.loads(run("inflatehd", stdin=json.dumps(d).encode()).stdout)
    assert i["cases"][0]["header_table_size"] == 256
    assert "header_table_size" not in i["cases"][1]
    # -S 1024: the deflater announces its own smaller maximum
    d = json.loads(run("deflatehd", ["-S", "1024"], stdin=json.dumps(STATIC_ONLY).encode()).stdout)
    assert d["cases"][0]["wire"] == "3fe107828684"
    # -s 100 -S 50: min announced first, then the current maximum
    r = HO.Deflater(50)
    r.change_table_size(100)
    want = r.deflate_block([(b":method", b"GET"), (b":scheme", b"http"), (b":path", b"/")]).hex()
    d = json.loads(run("deflatehd", ["-s", "100", "-S", "50"], stdin=json.dumps(STATIC_ONLY).encode()).stdout)
    assert d["cases"][0]["wire"] == want


def test_http1text_cpu():
    text = b":method: GET\n:scheme: https\n:path: /\n\n:status:   200\n\n:method: POST\n"
    d = json.loads(run("deflatehd", ["-t"], stdin=text).stdout)
    # the last block has no empty line after it and is dropped, as the reference does
    assert [c["wire"] for c in d["cases"]] == ["828784", "88"]
    assert headers_of(d["cases"][1]) == [(":status", "200")]


def test_driver_errors_cpu():
    p = run("deflatehd", stdin=b'{"nocases": []}', check=False)
    assert p.returncode != 0 and b"Missing 'cases' key" in p.stderr
    p = run("deflatehd", stdin=b"{", check=False)
    assert p.returncode != 0 and b"JSON loading failed" in p.stderr
    p = run("inflatehd", stdin=b'{"cases": [{"wire": "828"}]}', check=False)
    assert p.returncode != 0 and b"Badly formatted output value at 0" in p.stderr
    # a malformed block stops inflatehd after the cases before it
    p = run("inflatehd", stdin=b'{"cases": [{"wire": "82"}, {"wire": "80"}, {"wire": "82"}]}',
            check=False)
    assert p.returncode != 0 and b"inflate failed with error code -523 at 1" in p.stderr
    assert b'"seq": 0' in p.stdout and b'"seq": 1' not in p.stdout
    # cases the reference skips with a message
    p = run("deflatehd", stdin=b'{"cases": [1, {"x": 1}, {"headers": [{"a": 1}]}, '
                                b'{"headers": [{":method": "GET"}]}]}')
    doc = json.loads(p.stdout)
    assert [c["seq"] for c in doc["cases"]] == [3]
    assert b"Unexpected JSON type at 0" in p.stderr and b"'headers' key is missing at 1" in p.stderr
    assert b"value is not string at 2" in p.stderr


def test_config1_fixture_oracle():
    """The committed expected wire is the restated deflater's, and the
    restated inflater gets every header back from it."""
    cases = json.load(open(os.path.join(GOLD, "config1_cases.json")))
    gold = json.load(open(os.path.join(GOLD, "config1_wire.json")))
    assert len(cases["cases"]) == len(gold["wire"]) == 1000
    d, inf = HO.Deflater(), HO.Inflater()
    for c, w in zip(cases["cases"], gold["wire"]):
        hl = [(k.encode(), v.encode()) for k, v in headers_of(c)]
        assert d.deflate_block(hl).hex() == w
        st, f = inf.inflate_block(bytes.fromhex(w))
        assert [(n, v) for n, v, _ in f] == hl
    assert [[n.decode(), v.decode()] for n, v in d.table] == gold["final_table"]


# ---- GPU: literals ----
@pytest.mark.gpu
def test_config1_roundtrip(tmp_path):
    src = os.path.join(GOLD, "config1_cases.json")
    gold = json.load(open(os.path.join(GOLD, "config1_wire.json")))
    p = run("deflatehd", [src, "--timing"])
    d = json.loads(p.stdout)
    assert [c["wire"] for c in d["cases"]] == gold["wire"]
    cases = json.load(open(src))["cases"]
    for c, o in zip(cases, d["cases"]):
        assert headers_of(c) == headers_of(o)
        assert o["output_length"] == len(o["wire"]) // 2
    out = tmp_path / "wire.json"
    out.write_bytes(p.stdout)
    i = json.loads(run("inflatehd", [str(out)]).stdout)
    for c, o in zip(cases, i["cases"]):
        assert headers_of(c) == headers_of(o)
    assert "header_table_size" not in i["cases"][0]


@pytest.mark.gpu
@pytest.mark.parametrize("opts", [["-s", "256"], ["-S", "1024"], ["-s", "0"], ["-s", "8192", "-S", "2048"]])
def test_config1_table_sizes(opts):
    src = os.path.join(GOLD, "config1_cases.json")
    cases = json.load(open(src))["cases"][:300]
    doc = json.dumps({"cases": cases}).encode()
    s = int(opts[opts.index("-s") + 1]) if "-s" in opts else 4096
    S = int(opts[opts.index("-S") + 1]) if "-S" in opts else 4096
    r = HO.Deflater(S)
    if s != 4096:
        r.change_table_size(s)
    d = json.loads(run("deflatehd", opts + ["-d"], stdin=doc).stdout)
    inf = HO.Inflater()
    i = json.loads(run("inflatehd", ["-d"], stdin=json.dumps(d).encode()).stdout)
    for c, o, io in zip(cases, d["cases"], i["cases"]):
        hl = [(k.encode(), v.encode()) for k, v in headers_of(c)]
        assert o["wire"] == r.deflate_block(hl).hex()
        assert [(e["name"], e["value"]) for e in o["header_table"]["entries"]] == \
            [(n.decode(), v.decode()) for n, v in r.table]
        assert o["header_table"]["size"] == r.size
        # inflatehd's table is the deflater's, and so is the restated inflater's
        if "header_table_size" in o:
            inf.change_table_size(o["header_table_size"])
        inf.inflate_block(bytes.fromhex(o["wire"]))
        assert io["header_table"]["entries"] == o["header_table"]["entries"]
        assert io["header_table"]["max_size"] == inf.max
        assert headers_of(io) == headers_of(c)


@pytest.mark.gpu
def test_drivers_many_connections(tmp_path):
    """Several files = several connections in one batched call; each output
    equals the file run alone."""
    src = json.load(open(os.path.join(GOLD, "config1_cases.json")))["cases"]
    files = []
    for k in range(5):
        f = tmp_path / ("conn%d.json" % k)
        f.write_text(json.dumps({"cases": src[k * 150:(k + 1) * 150 + 17 * k]}))
        files.append(str(f))
    od = tmp_path / "out"
    od.mkdir()
    run("deflatehd", ["-o", str(od)] + files)
    wires = []
    for f in files:
        alone = run("deflatehd", [f]).stdout
        batched = (od / os.path.basename(f)).read_bytes()
        assert batched == alone
        wf = tmp_path / ("w_" + os.path.basename(f))
        wf.write_bytes(batched)
        wires.append(str(wf))
    oi = tmp_path / "inf"
    oi.mkdir()
    run("inflatehd", ["-o", str(oi)] + wires)
    for f, w in zip(files, wires):
        got = json.loads((oi / os.path.basename(w)).read_bytes())
        want = json.load(open(f))["cases"]
        assert [headers_of(c) for c in got["cases"]] == [headers_of(c) for c in want]
        assert (oi / os.path.basename(w)).read_bytes() == run("inflatehd", [w]).stdout
