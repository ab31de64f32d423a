// inflatehd -- batched HPACK decoder driver.
//
// Same input and output as the reference tool src/inflatehd.cc: an
// hpack-test-case JSON document ({"cases": [{"wire": hex,
// "header_table_size": N?}...]}) in; per case {seq, wire, headers,
// header_table_size when the maximum changed, header_table with -d} out,
// inside {"cases": [...]}.  Blocks are decoded as nghttp2_hd_inflate_hd3
// with in_final=1 then nghttp2_hd_inflate_end_headers (inflatehd.cc:97-173);
// a block that fails stops the program with "inflate failed with error code"
// as the reference does.
//
// What changes: the blocks of every input go through
// nghttp2_amd_hd_inflate_blocks, every Huffman literal of the batch decoded
// by one GPU call.  A batch is cut only where the reference's per-block
// bookkeeping needs the state in between: before a case whose
// header_table_size must be applied while earlier blocks of its connection
// are still pending, and after a block that starts with a table size update
// (its header_table_size output is the maximum after it).  Several input
// files are independent connections in the same batches (-o DIR writes
// DIR/<basename>).  -d decodes case by case.  --timing prints the wall time
// of the inflate calls to stderr as JSON.
#include <getopt.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <memory>
#include <string>
#include <vector>

#include "../../include/nghttp2_amd_hd.h"
#include "json_lite.h"

namespace {

struct Config {
  bool dump_table = false;
  bool timing = false;
  int repeat = 0;  // --repeat N: N more warm runs, best time reported
  std::string out_dir;
} cfg;

struct Case {
  int seq;
  const jl::Value *wire = nullptr;  // the input string, echoed back
  std::vector<uint8_t> bytes;
  bool has_size = false;
  size_t size = 0;
  bool comma_after = false;
  size_t old_max = 0, new_max = 0;  // max dynamic table size before / after
  int32_t status = 0;
  // the case's fields: nv[0..nnv) into arena (buffers of its batch call)
  const nghttp2_amd_hd_nv *nv = nullptr;
  size_t nnv = 0;
  const uint8_t *arena = nullptr;
  jl::Ptr table;
  bool done = false;
  bool skipped = false;  // header_table_size could not be applied
};

struct Conn {
  std::string path;
  jl::Ptr doc;
  std::vector<Case> cases;
  nghttp2_amd_hd_inflater *inf = nullptr;
};

void die(const std::string &m) {
  fprintf(stderr, "%s\n", m.c_str());
  exit(EXIT_FAILURE);
}

// to_ud / decode_hex (src/inflatehd.cc:58-73): letters are taken as hex
// digits by position, anything else as a decimal digit
uint8_t to_ud(char c) {
  if (c >= 'A' && c <= 'Z') return (uint8_t)(c - 'A' + 10);
  if (c >= 'a' && c <= 'z') return (uint8_t)(c - 'a' + 10);
  return (uint8_t)(c - '0');
}

// dump_inflate_header_table (src/comp_helper.c:66-96)
jl::Ptr dump_table(nghttp2_amd_hd_inflater *inf) {
  auto obj = jl::make(jl::Value::OBJ);
  auto ents = jl::make(jl::Value::ARR);
  const size_t n = nghttp2_amd_hd_inflate_get_num_table_entries(inf);
  for (size_t i = 62; i <= n; ++i) {
    const uint8_t *nm, *vl;
    size_t nl, vll;
    if (nghttp2_amd_hd_inflate_get_table_entry(inf, i, &nm, &nl, &vl, &vll) != 0) break;
    auto e = jl::make(jl::Value::OBJ);
    e->set("index", jl::integer((int64_t)i));
    e->set("name", jl::string(std::string((const char *)nm, nl)));
    e->set("value", jl::string(std::string((const char *)vl, vll)));
    e->set("size", jl::integer((int64_t)(nl + vll + 32)));
    ents->arr.push_back(e);
  }
  obj->set("entries", ents);
  obj->set("size", jl::integer((int64_t)nghttp2_amd_hd_inflate_get_dynamic_table_size(inf)));
  obj->set("max_size", jl::integer((int64_t)nghttp2_amd_hd_inflate_get_max_dynamic_table_size(inf)));
  return obj;
}

void read_json(Conn &c, const std::string &text) {
  jl::Reader r(text);
  c.doc = r.parse();
  if (!c.doc) die("JSON loading failed");
  const jl::Value *cases = c.doc->get("cases");
  if (!cases) die("Missing 'cases' key in root object");
  if (cases->kind != jl::Value::ARR) die("'cases' must be JSON array");
  const size_t len = cases->arr.size();
  for (size_t i = 0; i < len; ++i) {
    const jl::Value &obj = *cases->arr[i];
    if (obj.kind != jl::Value::OBJ) {
      fprintf(stderr, "Unexpected JSON type at %zu. It should be object.\n", i);
      continue;
    }
    Case k;
    k.seq = (int)i;
    k.wire = obj.get("wire");
    if (!k.wire) {
      fprintf(stderr, "'wire' key is missing at %zu\n", i);
      continue;
    }
    if (k.wire->kind != jl::Value::STR) {
      fprintf(stderr, "'wire' value is not string at %zu\n", i);
      continue;
    }
    if (const jl::Value *ts = obj.get("header_table_size")) {
      if (ts->kind != jl::Value::INT) {
        fprintf(stderr, "The value of 'header_table_size key' is not integer at %zu\n", i);
        continue;
      }
      k.has_size = true;
      k.size = (size_t)ts->i;
    }
    const std::string &w = k.wire->s;
    const size_t wl = strlen(w.c_str());
    if (wl & 1) {  // the reference exits here (inflatehd.cc:136-139)
      fprintf(stderr, "Badly formatted output value at %zu\n", i);
      exit(EXIT_FAILURE);
    }
    k.bytes.resize(wl / 2);
    for (size_t j = 0; j < wl; j += 2) k.bytes[j / 2] = (uint8_t)(to_ud(w[j]) << 4 | to_ud(w[j + 1]));
    k.comma_after = i + 1 < len;
    c.cases.push_back(std::move(k));
  }
}

// The buffers of every call of a run (the cases point into them).
struct CallBufs {
  std::unique_ptr<nghttp2_amd_hd_nv[]> nva;
  std::unique_ptr<uint8_t[]> arena;
};
std::vector<CallBufs> g_bufs;

// One batched inflate call over (connection, case) pairs; the caller's
// buffers grow until everything fits (a block that does not fit is not
// applied, so the rest is simply resubmitted).  Buffers are left
// uninitialised: the library writes what it reports.
double run_batch(std::vector<std::pair<Conn *, Case *>> &batch) {
  if (batch.empty()) return 0;
  const auto t0 = std::chrono::steady_clock::now();
  size_t wire = 0;
  for (auto &b : batch) wire += b.second->bytes.size();
  size_t nva_cap = wire + batch.size() + 16;
  size_t arena_cap = 16 * wire + 4096;
  size_t first = 0;
  std::vector<nghttp2_amd_hd_inflater *> infs;
  std::vector<const uint8_t *> ptrs;
  std::vector<size_t> lens;
  std::vector<int32_t> st;
  while (first < batch.size()) {
    const uint32_t nb = (uint32_t)(batch.size() - first);
    infs.resize(nb);
    ptrs.resize(nb);
    lens.resize(nb);
    st.resize(nb);
    for (uint32_t j = 0; j < nb; ++j) {
      infs[j] = batch[first + j].first->inf;
      ptrs[j] = batch[first + j].second->bytes.data();
      lens[j] = batch[first + j].second->bytes.size();
    }
    CallBufs cb;
    cb.nva.reset(new nghttp2_amd_hd_nv[nva_cap]);
    cb.arena.reset(new uint8_t[arena_cap]);
    size_t nv_used = 0, ar_used = 0;
    const int rv = nghttp2_amd_hd_inflate_blocks(infs.data(), nb, ptrs.data(), lens.data(), cb.nva.get(),
                                                 nva_cap, &nv_used, cb.arena.get(), arena_cap, &ar_used,
                                                 st.data(), nullptr);
    if (rv < 0 && rv != NGHTTP2_AMD_ERR_BUFFER_ERROR) die("inflate failed with error code " + std::to_string(rv));
    size_t f = 0;
    uint32_t j = 0;
    for (; j < nb && st[j] != NGHTTP2_AMD_ERR_BUFFER_ERROR; ++j) {
      Case &k = *batch[first + j].second;
      k.status = st[j];
      k.done = true;
      k.nv = cb.nva.get() + f;
      k.arena = cb.arena.get();
      while (f < nv_used && cb.nva[f].block == j) ++f;
      k.nnv = (size_t)(cb.nva.get() + f - k.nv);
    }
    g_bufs.push_back(std::move(cb));
    if (j == 0) {  // not even the first block fit
      nva_cap *= 2;
      arena_cap *= 2;
    }
    first += j;
  }
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

void usage() {
  printf(
      "HPACK HTTP/2 header decoder (batched; GPU Huffman decode)\n"
      "Usage: inflatehd [OPTIONS] [FILE...] < INPUT\n\n"
      "Reads hpack-test-case JSON with \"wire\" hex blocks from FILEs or stdin;\n"
      "each FILE is its own compression context.  Prints the inflated fields.\n\n"
      "OPTIONS:\n"
      "    -d, --dump-header-table    output the dynamic table after each case\n"
      "    -o, --output-dir=<DIR>     write FILE's output to DIR/<basename FILE>\n"
      "        --timing               inflate wall time to stderr (JSON)\n"
      "        --repeat=<N>           N more warm runs (fresh contexts); best in warm_seconds\n");
}

}  // namespace

int main(int argc, char **argv) {
  static const struct option longopts[] = {{"dump-header-table", no_argument, nullptr, 'd'},
                                           {"output-dir", required_argument, nullptr, 'o'},
                                           {"timing", no_argument, nullptr, 'T'},
                                           {"repeat", required_argument, nullptr, 'R'},
                                           {"help", no_argument, nullptr, 'h'},
                                           {nullptr, 0, nullptr, 0}};
  for (;;) {
    const int c = getopt_long(argc, argv, "dho:", longopts, nullptr);
    if (c == -1) break;
    switch (c) {
      case 'h': usage(); return 0;
      case 'd': cfg.dump_table = true; break;
      case 'o': cfg.out_dir = optarg; break;
      case 'T': cfg.timing = true; break;
      case 'R': cfg.repeat = atoi(optarg); break;
      default: return EXIT_FAILURE;
    }
  }
  std::vector<Conn> conns;
  if (optind >= argc) {
    conns.emplace_back();
  } else {
    for (int i = optind; i < argc; ++i) {
      conns.emplace_back();
      conns.back().path = argv[i];
    }
  }
  if (conns.size() > 1 && cfg.out_dir.empty()) die("several inputs need -o DIR");
  for (auto &c : conns) {
    std::string text;
    FILE *f = c.path.empty() ? stdin : fopen(c.path.c_str(), "rb");
    if (!f || !jl::read_file(f, text)) die("cannot read " + (c.path.empty() ? std::string("stdin") : c.path));
    if (f != stdin) fclose(f);
    read_json(c, text);
  }

  // ---- batches, connections interleaved case by case
  size_t nblocks = 0, wire_bytes = 0, fields = 0;
  auto run_all = [&]() -> double {  // fresh inflaters, every case decoded once
    double secs = 0;
    nblocks = wire_bytes = 0;
    g_bufs.clear();
    for (auto &c : conns) {
      if (c.inf) nghttp2_amd_hd_inflate_del(c.inf);
      if (nghttp2_amd_hd_inflate_new(&c.inf) != 0) die("inflate_new failed");
      for (auto &k : c.cases) {
        k.nv = nullptr;
        k.nnv = 0;
        k.status = 0;
        k.done = k.skipped = false;
        k.table.reset();
      }
    }
    std::vector<std::pair<Conn *, Case *>> batch;
    std::vector<char> pending(conns.size(), 0);
    auto flush = [&]() {
      secs += run_batch(batch);
      batch.clear();
      std::fill(pending.begin(), pending.end(), 0);
    };
    size_t maxcases = 0;
    for (auto &c : conns) maxcases = std::max(maxcases, c.cases.size());
    for (size_t r = 0; r < maxcases; ++r)
      for (size_t ci = 0; ci < conns.size(); ++ci) {
        Conn &c = conns[ci];
        if (r >= c.cases.size()) continue;
        Case &k = c.cases[r];
        if (k.has_size && pending[ci]) flush();
        k.old_max = nghttp2_amd_hd_inflate_get_max_dynamic_table_size(c.inf);
        if (k.has_size) {
          const int rv = nghttp2_amd_hd_inflate_change_table_size(c.inf, k.size);
          if (rv != 0) {
            fprintf(stderr, "nghttp2_hd_change_table_size() failed with error %d at %d\n", rv, k.seq);
            k.skipped = true;  // no output for it (the reference's return -1)
            continue;
          }
        }
        // a block without a size update keeps the maximum set so far
        k.new_max = nghttp2_amd_hd_inflate_get_max_dynamic_table_size(c.inf);
        batch.emplace_back(&c, &k);
        pending[ci] = 1;
        nblocks++;
        wire_bytes += k.bytes.size();
        const bool size_update = !k.bytes.empty() && (k.bytes[0] & 0xE0) == 0x20;
        if (size_update || cfg.dump_table) {
          flush();
          k.new_max = nghttp2_amd_hd_inflate_get_max_dynamic_table_size(c.inf);
          if (cfg.dump_table) k.table = dump_table(c.inf);
        }
      }
    flush();
    return secs;
  };
  const double secs = run_all();
  double warm = -1;
  for (int r = 0; r < cfg.repeat; ++r) {
    const double t = run_all();
    if (warm < 0 || t < warm) warm = t;
  }

  // ---- outputs (to_json, src/inflatehd.cc:75-95)
  for (auto &c : conns) {
    std::string o = "{\n  \"cases\":\n  [\n";
    bool failed = false;
    for (auto &k : c.cases) {
      if (k.skipped) continue;
      if (k.status < 0) {
        fprintf(stderr, "inflate failed with error code %d at %d\n", k.status, k.seq);
        failed = true;
        break;
      }
      auto obj = jl::make(jl::Value::OBJ);
      obj->set("seq", jl::integer(k.seq));
      obj->set("wire", jl::string(k.wire->s));
      auto hs = jl::make(jl::Value::ARR);
      for (size_t q = 0; q < k.nnv; ++q) {
        const nghttp2_amd_hd_nv &f = k.nv[q];
        auto p = jl::make(jl::Value::OBJ);
        // the name as a C string, as dump_header (src/comp_helper.c:98-110) takes it
        p->set(std::string((const char *)k.arena + f.name_off),
               jl::string(std::string((const char *)k.arena + f.value_off, f.value_len)));
        hs->arr.push_back(p);
      }
      fields += k.nnv;
      obj->set("headers", hs);
      if (k.old_max != k.new_max) obj->set("header_table_size", jl::integer((int64_t)k.new_max));
      if (k.table) obj->set("header_table", k.table);
      jl::dump(o, *obj, 0);
      o += "\n";
      if (k.comma_after) o += ",\n";
    }
    if (!failed) o += "  ]\n}\n";
    FILE *f = stdout;
    if (!cfg.out_dir.empty()) {
      const size_t sl = c.path.find_last_of('/');
      const std::string base =
          c.path.empty() ? "stdin.json" : (sl == std::string::npos ? c.path : c.path.substr(sl + 1));
      f = fopen((cfg.out_dir + "/" + base).c_str(), "wb");
      if (!f) die("cannot write " + cfg.out_dir + "/" + base);
    }
    fwrite(o.data(), 1, o.size(), f);
    if (f != stdout) fclose(f);
    if (failed) exit(EXIT_FAILURE);
  }
  for (auto &c : conns) nghttp2_amd_hd_inflate_del(c.inf);
  if (cfg.timing)
    fprintf(stderr,
            "{\"timing\": {\"connections\": %zu, \"blocks\": %zu, \"fields\": %zu, \"wire_bytes\": %zu, "
            "\"seconds\": %.6f, \"warm_seconds\": %.6f, \"per_case_calls\": %s}}\n",
            conns.size(), nblocks, fields, wire_bytes, secs, warm, cfg.dump_table ? "true" : "false");
  return 0;
}
