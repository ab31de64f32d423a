// deflatehd -- batched HPACK encoder driver.
//
// Same input and output as the reference tool src/deflatehd.cc: an
// hpack-test-case JSON document ({"cases": [{"headers": [{name: value}...]}]})
// or, with -t, HTTP/1-style header blocks separated by an empty line, in;
// one JSON object per case out (seq, input_length, output_length,
// percentage_of_original_size, wire hex, headers, header_table_size at seq 0,
// header_table with -d), inside {"cases": [...]}, and the stderr line
// "Overall: input= output= ratio=".  Options -s/-S/-d/-t as the reference's
// (deflatehd.cc:366-388).
//
// What changes: every case of every input goes through ONE
// nghttp2_amd_hd_deflate_blocks call (one GPU emit_strings batch for all
// literals) instead of one nghttp2_hd_deflate_hd2 per case.  Several input
// files are several independent connections (one deflater each) in that same
// call; with -o DIR each file's output goes to DIR/<basename>.  -d needs the
// table after each case, so it deflates case by case.  --timing prints the
// batched call's wall time to stderr as JSON.
#include <getopt.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

#include "../../include/nghttp2_amd_hd.h"
#include "json_lite.h"

namespace {

struct Config {
  size_t table_size = 4096;          // -s  SETTINGS_HEADER_TABLE_SIZE
  size_t deflate_table_size = 4096;  // -S  deflater's own maximum
  bool http1text = false;            // -t
  bool dump_table = false;           // -d
  bool timing = false;               // --timing
  int repeat = 0;                    // --repeat N: N more warm runs, best reported
  std::string out_dir;               // -o
} cfg;

// One header list read from the input.
struct Case {
  int seq;
  std::vector<nghttp2_amd_nv> nva;
  size_t inputlen = 0;
  bool comma_after = false;  // the reference prints "," after case i when i+1 < len
  uint32_t block = 0;        // index in the batch
};

struct Conn {
  std::string path;  // "" = stdin
  jl::Ptr doc;
  std::vector<std::string> owned;  // -t strings
  std::vector<Case> cases;
  nghttp2_amd_hd_deflater *d = nullptr;
  bool leading_comma = false;  // -t prints "," before blocks after the first
};

size_t input_sum, output_sum;

void die(const std::string &m) {
  fprintf(stderr, "%s\n", m.c_str());
  exit(EXIT_FAILURE);
}

std::string hex(const uint8_t *p, size_t n) {
  static const char h[] = "0123456789abcdef";
  std::string s(n * 2, '0');
  for (size_t i = 0; i < n; ++i) {
    s[2 * i] = h[p[i] >> 4];
    s[2 * i + 1] = h[p[i] & 15];
  }
  return s;
}

jl::Ptr dump_headers(const std::vector<nghttp2_amd_nv> &nva) {
  auto a = jl::make(jl::Value::ARR);
  for (auto &nv : nva) {
    auto o = jl::make(jl::Value::OBJ);
    o->set(std::string((const char *)nv.name, nv.namelen),
           jl::string(std::string((const char *)nv.value, nv.valuelen)));
    a->arr.push_back(o);
  }
  return a;
}

// dump_deflate_header_table (src/comp_helper.c:34-64)
jl::Ptr dump_table(nghttp2_amd_hd_deflater *d) {
  auto obj = jl::make(jl::Value::OBJ);
  auto ents = jl::make(jl::Value::ARR);
  const size_t n = nghttp2_amd_hd_deflate_get_num_table_entries(d);
  for (size_t i = 62; i <= n; ++i) {
    const uint8_t *nm, *vl;
    size_t nl, vll;
    if (nghttp2_amd_hd_deflate_get_table_entry(d, i, &nm, &nl, &vl, &vll) != 0) break;
    auto e = jl::make(jl::Value::OBJ);
    e->set("index", jl::integer((int64_t)i));
    e->set("name", jl::string(std::string((const char *)nm, nl)));
    e->set("value", jl::string(std::string((const char *)vl, vll)));
    e->set("size", jl::integer((int64_t)(nl + vll + 32)));
    ents->arr.push_back(e);
  }
  obj->set("entries", ents);
  obj->set("size", jl::integer((int64_t)nghttp2_amd_hd_deflate_get_dynamic_table_size(d)));
  obj->set("max_size", jl::integer((int64_t)nghttp2_amd_hd_deflate_get_max_dynamic_table_size(d)));
  return obj;
}

// output_to_json (src/deflatehd.cc:80-117)
void case_json(std::string &o, const Case &c, const uint8_t *wire, size_t len, jl::Ptr table) {
  auto obj = jl::make(jl::Value::OBJ);
  obj->set("seq", jl::integer(c.seq));
  obj->set("input_length", jl::integer((int64_t)c.inputlen));
  obj->set("output_length", jl::integer((int64_t)len));
  obj->set("percentage_of_original_size",
           jl::real(c.inputlen == 0 ? 0.0 : (double)len / (double)c.inputlen * 100));
  obj->set("wire", jl::string(hex(wire, len)));
  obj->set("headers", dump_headers(c.nva));
  if (c.seq == 0) obj->set("header_table_size", jl::integer((int64_t)cfg.table_size));
  if (table) obj->set("header_table", table);
  jl::dump(o, *obj, 0);
  o += "\n";
}

// deflate_hd_json (src/deflatehd.cc:137-186): the cases of one document
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
    const jl::Value *hs = obj.get("headers");
    if (!hs) {
      fprintf(stderr, "'headers' key is missing at %zu\n", i);
      continue;
    }
    if (hs->kind != jl::Value::ARR) {
      fprintf(stderr, "The value of 'headers' key must be an array at %zu\n", i);
      continue;
    }
    Case k;
    k.seq = (int)i;
    bool ok = true;
    for (auto &pair : hs->arr) {
      if (pair->kind != jl::Value::OBJ || pair->obj.size() != 1) {
        fprintf(stderr, "bad formatted name/value pair object at %zu\n", i);
        ok = false;
        break;
      }
      const auto &kv = pair->obj[0];
      if (kv.second->kind != jl::Value::STR) {
        fprintf(stderr, "value is not string at %zu\n", i);
        ok = false;
        break;
      }
      nghttp2_amd_nv nv;
      nv.name = (const uint8_t *)kv.first.c_str();
      nv.namelen = strlen(kv.first.c_str());  // C strings, as jansson hands them over
      nv.value = (const uint8_t *)kv.second->s.c_str();
      nv.valuelen = strlen(kv.second->s.c_str());
      nv.flags = 0;
      k.inputlen += nv.namelen + nv.valuelen;
      k.nva.push_back(nv);
    }
    if (!ok) continue;
    k.comma_after = i + 1 < len;
    c.cases.push_back(std::move(k));
  }
}

// perform_from_http1text (src/deflatehd.cc:247-313): "name: value" lines,
// one empty line after each block; a block not followed by one is dropped,
// as the reference drops it.
void read_http1(Conn &c, const std::string &text) {
  c.leading_comma = true;
  size_t pos = 0;
  std::vector<std::pair<std::string, std::string>> cur;
  std::vector<std::vector<std::pair<std::string, std::string>>> blocks;
  while (pos < text.size()) {
    const size_t eol = text.find('\n', pos);
    const bool last = eol == std::string::npos;
    const std::string line = text.substr(pos, last ? std::string::npos : eol - pos);
    pos = last ? text.size() : eol + 1;
    if (line.empty()) {  // an empty line ends the block
      blocks.push_back(cur);
      cur.clear();
      continue;
    }
    const size_t colon = line.find(':', 1);
    if (colon == std::string::npos)
      die("Bad HTTP/1 header field format at " + std::to_string(blocks.size()) + ".");
    size_t v = colon + 1;
    while (v < line.size() && (line[v] == ' ' || line[v] == '\t')) ++v;
    size_t ve = v;
    while (ve < line.size() && line[ve] != '\r') ++ve;
    cur.emplace_back(line.substr(0, colon), line.substr(v, ve - v));
  }
  size_t total = 0;
  for (auto &b : blocks) total += 2 * b.size();
  c.owned.reserve(total);  // the strings must not move once pointed at
  int seq = 0;
  for (auto &b : blocks) {
    Case k;
    k.seq = seq++;
    for (auto &f : b) {
      c.owned.push_back(f.first);
      const std::string &n = c.owned.back();
      c.owned.push_back(f.second);
      const std::string &val = c.owned.back();
      nghttp2_amd_nv nv{(const uint8_t *)n.c_str(), (const uint8_t *)val.c_str(), strlen(n.c_str()),
                        strlen(val.c_str()), 0};
      k.inputlen += nv.namelen + nv.valuelen;
      k.nva.push_back(nv);
    }
    c.cases.push_back(std::move(k));
  }
}

// init_deflater (src/deflatehd.cc:188-195)
nghttp2_amd_hd_deflater *init_deflater() {
  nghttp2_amd_hd_deflater *d = nullptr;
  if (nghttp2_amd_hd_deflate_new(&d, cfg.deflate_table_size) != 0) die("deflate_new failed");
  if (cfg.table_size != 4096) nghttp2_amd_hd_deflate_change_table_size(d, cfg.table_size);
  return d;
}

void usage() {
  printf(
      "HPACK HTTP/2 header encoder (batched; GPU string literals)\n"
      "Usage: deflatehd [OPTIONS] [FILE...] < INPUT\n\n"
      "Reads hpack-test-case JSON (or, with -t, HTTP/1-style header blocks each\n"
      "followed by an empty line) from FILEs or stdin; each FILE is its own\n"
      "compression context.  Prints the deflated blocks as JSON.\n\n"
      "OPTIONS:\n"
      "    -t, --http1text            HTTP/1 style header field text input\n"
      "    -s, --table-size=<N>       SETTINGS_HEADER_TABLE_SIZE (default 4096)\n"
      "    -S, --deflate-table-size=<N>  use the first N bytes of the table (4096)\n"
      "    -d, --dump-header-table    output the dynamic table after each case\n"
      "    -o, --output-dir=<DIR>     write FILE's output to DIR/<basename FILE>\n"
      "        --timing               batched call wall time to stderr (JSON)\n"
      "        --repeat=<N>           N more warm runs (fresh contexts); best in warm_seconds\n");
}

}  // namespace

int main(int argc, char **argv) {
  static const struct option longopts[] = {{"http1text", no_argument, nullptr, 't'},
                                           {"table-size", required_argument, nullptr, 's'},
                                           {"deflate-table-size", required_argument, nullptr, 'S'},
                                           {"dump-header-table", no_argument, nullptr, 'd'},
                                           {"output-dir", required_argument, nullptr, 'o'},
                                           {"timing", no_argument, nullptr, 'T'},
                                           {"repeat", required_argument, nullptr, 'R'},
                                           {"help", no_argument, nullptr, 'h'},
                                           {nullptr, 0, nullptr, 0}};
  for (;;) {
    const int c = getopt_long(argc, argv, "S:dhs:to:", longopts, nullptr);
    if (c == -1) break;
    char *end = nullptr;
    switch (c) {
      case 'h': usage(); return 0;
      case 't': cfg.http1text = true; break;
      case 's':
        cfg.table_size = strtoull(optarg, &end, 10);
        if (!*optarg || *end) die("-s: Bad option value");
        break;
      case 'S':
        cfg.deflate_table_size = strtoull(optarg, &end, 10);
        if (!*optarg || *end) die("-S: Bad option value");
        break;
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
    if (cfg.http1text) read_http1(c, text);
    else read_json(c, text);
    c.d = init_deflater();
  }

  // ---- the batch: every case of every connection, connections interleaved
  // case by case (only the order within a connection matters)
  std::vector<nghttp2_amd_hd_deflater *> defl;
  std::vector<nghttp2_amd_nv> nva;
  std::vector<uint32_t> nv_off{0};
  std::vector<size_t> block_conn;
  size_t bound = 0, maxcases = 0;
  for (auto &c : conns) maxcases = std::max(maxcases, c.cases.size());
  for (size_t r = 0; r < maxcases; ++r)
    for (auto &c : conns) {
      if (r >= c.cases.size()) continue;
      Case &k = c.cases[r];
      k.block = (uint32_t)defl.size();
      defl.push_back(c.d);
      block_conn.push_back(&c - conns.data());
      nva.insert(nva.end(), k.nva.begin(), k.nva.end());
      nv_off.push_back((uint32_t)nva.size());
      bound += nghttp2_amd_hd_deflate_bound(c.d, k.nva.data(), k.nva.size());
    }
  const uint32_t nb = (uint32_t)defl.size();
  std::vector<uint8_t> out(bound + 1);
  std::vector<uint32_t> out_off(nb + 1, 0);
  std::vector<int32_t> status(nb, 0);
  std::vector<jl::Ptr> tables(nb);

  const auto t0 = std::chrono::steady_clock::now();
  if (!cfg.dump_table) {
    const int rv = nghttp2_amd_hd_deflate_blocks(defl.data(), nb, nva.data(), nv_off.data(), out.data(),
                                                 out.size(), out_off.data(), status.data(), nullptr);
    if (rv < 0 && rv != NGHTTP2_AMD_ERR_BUFFER_ERROR) die("deflate failed with error code " + std::to_string(rv));
  } else {
    size_t o = 0;
    for (uint32_t b = 0; b < nb; ++b) {
      const uint32_t loc[2] = {0, nv_off[b + 1] - nv_off[b]};
      uint32_t off2[2];
      int32_t st;
      const int rv = nghttp2_amd_hd_deflate_blocks(&defl[b], 1, nva.data() + nv_off[b], loc, out.data() + o,
                                                   out.size() - o, off2, &st, nullptr);
      if (rv < 0 && rv != NGHTTP2_AMD_ERR_BUFFER_ERROR) die("deflate failed with error code " + std::to_string(rv));
      status[b] = st;
      out_off[b] = (uint32_t)o;
      o += off2[1];
      out_off[b + 1] = (uint32_t)o;
      tables[b] = dump_table(defl[b]);
    }
  }
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  double warm = -1;
  if (!cfg.dump_table && cfg.repeat > 0) {  // warm runs: fresh deflaters, same batch
    std::vector<uint8_t> out2(out.size());
    std::vector<uint32_t> off2(nb + 1);
    std::vector<int32_t> st2(nb);
    for (int r = 0; r < cfg.repeat; ++r) {
      std::vector<nghttp2_amd_hd_deflater *> fresh(conns.size());
      for (auto &f : fresh) f = init_deflater();
      std::vector<nghttp2_amd_hd_deflater *> d2(nb);
      for (uint32_t b = 0; b < nb; ++b) d2[b] = fresh[block_conn[b]];
      const auto t1 = std::chrono::steady_clock::now();
      const int rv = nghttp2_amd_hd_deflate_blocks(d2.data(), nb, nva.data(), nv_off.data(), out2.data(),
                                                   out2.size(), off2.data(), st2.data(), nullptr);
      const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
      if (rv < 0 || off2 != out_off || memcmp(out2.data(), out.data(), out_off[nb]) != 0)
        die("warm run differs from the first run");
      if (warm < 0 || t < warm) warm = t;
      for (auto f : fresh) nghttp2_amd_hd_deflate_del(f);
    }
  }

  // ---- outputs, per connection in case order
  for (auto &c : conns) {
    std::string o = "{\n  \"cases\":\n  [\n";
    bool failed = false;
    for (size_t r = 0; r < c.cases.size(); ++r) {
      const Case &k = c.cases[r];
      const int32_t st = status[k.block];
      if (st < 0) {  // deflate_hd (src/deflatehd.cc:124-129): report and stop
        fprintf(stderr, "deflate failed with error code %d at %d\n", st, k.seq);
        failed = true;
        break;
      }
      if (c.leading_comma && r > 0) o += ",\n";
      const uint32_t a = out_off[k.block], b = out_off[k.block + 1];
      input_sum += k.inputlen;
      output_sum += b - a;
      case_json(o, k, out.data() + a, b - a, tables[k.block]);
      if (!c.leading_comma && k.comma_after) o += ",\n";
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
  for (auto &c : conns) nghttp2_amd_hd_deflate_del(c.d);

  fflush(stdout);
  fprintf(stderr, "Overall: input=%zu output=%zu ratio=%.2f\n", input_sum, output_sum,
          input_sum == 0 ? 0.0 : (double)output_sum / (double)input_sum);
  if (cfg.timing)
    fprintf(stderr,
            "{\"timing\": {\"connections\": %zu, \"blocks\": %u, \"fields\": %zu, \"input_bytes\": %zu, "
            "\"wire_bytes\": %zu, \"seconds\": %.6f, \"warm_seconds\": %.6f, \"per_case_calls\": %s}}\n",
            conns.size(), nb, nva.size(), input_sum, output_sum, secs, warm, cfg.dump_table ? "true" : "false");
  return 0;
}
