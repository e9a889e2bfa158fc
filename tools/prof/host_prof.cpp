// host_prof.cpp — CPU timing of the drop-in host layer without a device:
// Columnarize and Apply (outputs synthesised: every other trace kept, every
// templated span given "/t/{id}") over a JSON array of Traces, per phase.
// Diagnostics only; links the product library.
//   g++ -O2 -std=c++17 -Iodigos_amd/csrc -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ tools/prof/host_prof.cpp
//       -Lodigos_amd/_lib -lodigos_amd -Wl,-rpath,$PWD/odigos_amd/_lib -o /tmp/host_prof
//   /tmp/host_prof cfg.json traces.json reps [keep_mod]
#include <chrono>
#include <cstring>
#include <cstdio>
#include <fstream>
#include <sstream>

#include "host.hpp"
#include "json.hpp"

using namespace ose;
static std::string slurp(const char* f) {
  std::ifstream in(f);
  std::stringstream ss;
  ss << in.rdbuf();
  return ss.str();
}
int main(int argc, char** argv) {
  if (argc < 4) return 2;
  TracesProcessor tp(ProcKind::Pipeline, parse_json(slurp(argv[1])));
  if (!tp.error().empty()) { fprintf(stderr, "%s\n", tp.error().c_str()); return 1; }
  tp.group_mode = OSE_GROUP_TRACE_ID;
  Json arr = parse_json(slurp(argv[2]));
  std::vector<Traces> items;
  for (auto& t : arr.arr) items.push_back(traces_from_json(t));
  const int reps = atoi(argv[3]);
  const uint64_t keep_mod = argc > 4 ? strtoull(argv[4], nullptr, 0) : 2;   // keep one trace in keep_mod
  std::vector<Traces> work;
  for (int r = 0; r < reps; r++)
    for (auto& t : items) work.push_back(t);
  using clk = std::chrono::steady_clock;
  double tc = 0, ta = 0;
  size_t spans = 0;
  const char tmpl[] = "/t/{id}";
  for (auto& td : work) {
    auto a = clk::now();
    auto hb = tp.Columnarize(td);
    auto b = clk::now();
    const uint64_t n = hb->cols.n_spans;
    spans += n;
    // templates as long as the paths (the span's own path bytes, copied into
    // the template arena: heap-sized strings like real templates), renames
    // where the span's name is its method
    size_t need = 16;
    for (uint64_t i = 0; i < n; i++) need += hb->path[i].len;
    if (hb->tmpl_arena.size() < need + 16) { hb->tmpl_arena.resize(need + 16); hb->bind(); }
    uint32_t at = 0;
    for (uint64_t i = 0; i < n; i++) {
      hb->outs.keep[i] = (uint8_t)(((hb->trace_id[2 * i] >> 7) % keep_mod) == 0);
      const bool has_path = (hb->url_flags[i] & OSE_URL_PATH_MASK) != 0;
      hb->outs.url_out[i] = has_path ? (uint8_t)(OSE_OUT_SET_ATTR | ((hb->url_flags[i] & OSE_URL_NAME_EQ_METHOD) ? OSE_OUT_RENAME : 0)) : 0;
      const ose_strref pr = hb->path[i];
      if (pr.len) memcpy(hb->outs.tmpl_arena + at, hb->arena.data() + pr.off, pr.len);
      hb->outs.tmpl[i] = has_path && pr.len ? ose_strref{at, pr.len} : ose_strref{0, 7};
      at += pr.len;
    }
    (void)tmpl;
    auto c = clk::now();
    tp.Apply(*hb, td);
    auto d = clk::now();
    tc += std::chrono::duration<double>(b - a).count();
    ta += std::chrono::duration<double>(d - c).count();
  }
  printf("calls %zu spans %zu columnarize %.1f us/call (%.1f ns/span) apply %.1f us/call (%.1f ns/span)\n", work.size(),
         spans, tc / work.size() * 1e6, tc / spans * 1e9, ta / work.size() * 1e6, ta / spans * 1e9);
  return 0;
}
