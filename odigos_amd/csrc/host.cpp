// host.cpp — see host.hpp.  Columnarisation mirrors what each reference
// function reads from pdata; Apply mirrors what it writes.
#include "host.hpp"

#include "columnize.hpp"
#include "otlp_pb.hpp"

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstring>
#include <map>
#include <set>
#include <string_view>
#include <thread>

#include "span_attr.hpp"
#include "taskpool.hpp"
#include "urlparse.hpp"

namespace ose {

std::map<std::string, uint32_t> intern_services(const SamplingConfig& c) {
  std::map<std::string, uint32_t> m;
  auto add = [&](const std::string& s) { if (!m.count(s)) m.emplace(s, (uint32_t)m.size()); };
  for (auto* lvl : {&c.global_rules, &c.service_rules, &c.endpoint_rules})
    for (auto& r : *lvl) {
      if (r.rtype == RuleType::HttpLatency) add(r.latency.service_name);
      if (r.rtype == RuleType::ServiceName) add(r.service.service_name);
      if (r.rtype == RuleType::SpanAttribute) add(r.attr.service_name);
    }
  return m;
}

void HostBatch::bind() {
  cols.arena = arena.data();
  cols.trace_id = trace_id.data();
  cols.start_ns = start.data();
  cols.end_ns = end.data();
  cols.status = status.data();
  cols.kind = kind.data();
  cols.resource = resource.data();
  cols.scope = scope.data();
  cols.url_flags = url_flags.data();
  cols.path = path.data();
  cols.route = route.data();
  cols.span_size = span_size.data();
  cols.name_len = name_len.data();
  cols.res_svc = res_svc.data();
  cols.res_svc_str = res_svc_str.data();
  cols.res_url_ok = res_url_ok.data();
  cols.res_attrset = res_attrset.data();
  cols.res_size = res_size.data();
  cols.scope_size = scope_size.data();
  cols.scope_resource = scope_resource.data();
  cols.attr_match = attr_match.data();
  cols.attr_match_words = attr_words;
  cols.attr_type = cols.n_attr_keys ? attr_type.data() : nullptr;
  cols.attr_val = cols.n_attr_keys ? attr_val.data() : nullptr;
  outs.keep = keep.data();
  outs.trace_count = trace_count.data();
  outs.trace_first_span = trace_first_span.data();
  outs.trace_keep = trace_keep.data();
  outs.trace_level = trace_level.data();
  outs.trace_ratio = trace_ratio.data();
  outs.url_out = url_out.data();
  outs.tmpl = tmpl.data();
  outs.tmpl_arena = tmpl_arena.data();
  outs.tmpl_arena_cap = tmpl_arena.size() - 16;
  outs.tmpl_arena_used = tmpl_used.data();
  outs.attrset_bytes = attrset_bytes.data();
  outs.accepted_spans = accepted.data();
  outs.res_bytes = res_bytes.data();
  outs.device_status = device_status.data();
}

namespace {

const char* kProcType[] = {"odigossampling", "odigosurltemplate", "odigostrafficmetrics", "pipeline"};

}  // namespace

TracesProcessor::TracesProcessor(ProcKind k, const Json& cfg) : kind_(k), cfg_json_(cfg) {
  Json c = cfg.is_null() ? Json::object() : cfg;
  switch (k) {
    case ProcKind::Sampling: err_ = decode_sampling_config(c, sampling_); has_sampling_ = true; break;
    case ProcKind::UrlTemplate: err_ = decode_url_config(c, url_); has_url_ = true; break;
    case ProcKind::TrafficMetrics: err_ = decode_traffic_config(c, traffic_); has_traffic_ = true; break;
    case ProcKind::Pipeline:
      if (const Json* j = c.get("odigossampling")) { err_ = decode_sampling_config(*j, sampling_); has_sampling_ = true; }
      if (err_.empty()) if (const Json* j = c.get("odigosurltemplate")) { err_ = decode_url_config(*j, url_); has_url_ = true; }
      if (err_.empty()) if (const Json* j = c.get("odigostrafficmetrics")) { err_ = decode_traffic_config(*j, traffic_); has_traffic_ = true; }
      group_mode = OSE_GROUP_TRACE_ID;
      break;
  }
  // span_attribute conditions: compiled here (json ones run in the walk);
  // newUrlTemplateProcessor's errors are decode_url_config's (factory.go:37-40)
  if (err_.empty())
    err_ = ctx_.build(has_url_ ? &url_ : nullptr, has_sampling_ ? &sampling_ : nullptr, has_traffic_ ? &traffic_ : nullptr);
}

TracesProcessor::~TracesProcessor() {
  if (eng_) ose_engine_destroy(eng_);
}

uint32_t TracesProcessor::stages() const {
  return (has_sampling_ ? OSE_STAGE_SAMPLE : 0) | (has_url_ ? OSE_STAGE_TEMPLATE : 0) | (has_traffic_ ? OSE_STAGE_SIZE : 0);
}

int TracesProcessor::ensure_engine() {   // callers hold mu_
  if (eng_) return 0;
  Json root = Json::object();
  if (kind_ == ProcKind::Pipeline) root = cfg_json_;
  else root.set(kProcType[(int)kind_], cfg_json_.is_null() ? Json::object() : cfg_json_);
  std::string s;
  dump_json(s, root);
  return ose_engine_create(s.c_str(), &eng_);
}

double TracesProcessor::next_uniform() {
  // splitmix64 stream -> [0,1)
  uint64_t z = (seed_ += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  draws_++;
  return (double)(z >> 11) * 0x1.0p-53;
}

// The columns of a batch: presized, then filled by resource ranges in
// parallel on the host task pool (taskpool.hpp) when the batch is large
// enough to pay for it.  Each range writes its spans' columns in place and
// its strings into a range-local arena and interns its attribute sets
// locally; the merge concatenates the arenas (shifting the ranges' string
// refs) and renumbers the attribute sets in first-appearance order, so the
// result is the one a sequential walk gives.  keep_copy: the batch keeps a
// copy of the traces (the test seam's apply reads it); ProcessTraces
// applies the outputs to its own traces and passes false.
std::unique_ptr<HostBatch> TracesProcessor::Columnarize(const Traces& td, bool keep_copy) const {
  auto hb = std::make_unique<HostBatch>();
  if (keep_copy) hb->td = td;
  const Traces& t = keep_copy ? hb->td : td;
  const size_t R = t.resource_spans.size();
  std::vector<uint64_t> span0(R + 1, 0), scope0(R + 1, 0);
  for (size_t ri = 0; ri < R; ri++) {
    uint64_t ns = 0;
    for (auto& ss : t.resource_spans[ri].scope_spans) ns += ss.spans.size();
    span0[ri + 1] = span0[ri] + ns;
    scope0[ri + 1] = scope0[ri] + t.resource_spans[ri].scope_spans.size();
  }
  const size_t N = span0[R], S = scope0[R];
  const size_t nk = ctx_.attr_plan.keys.size(), W = std::max<size_t>(1, (ctx_.attr_preds.size() + 63) / 64);
  hb->trace_id.resize(2 * N);
  hb->start.resize(N);
  hb->end.resize(N);
  hb->status.resize(N);
  hb->kind.resize(N);
  hb->resource.resize(N);
  hb->scope.resize(N);
  hb->span_size.resize(N);
  hb->name_len.resize(N);
  hb->url_flags.resize(N);
  hb->path.resize(N);
  hb->route.resize(N);
  hb->attr_match.assign(W * N, 0);   // word-major (ose_columns.attr_match_words)
  hb->attr_words = (uint32_t)W;
  hb->attr_type.resize(nk * N);      // key-major
  hb->attr_val.resize(nk * N);
  hb->res_svc.resize(R);
  hb->res_svc_str.resize(R);
  hb->res_url_ok.resize(R);
  hb->res_attrset.resize(R);
  hb->res_size.resize(R);
  hb->scope_size.resize(S);
  hb->scope_resource.resize(S);
  using AttrSet = std::vector<std::pair<std::string, std::string>>;
  struct Range {
    size_t r0 = 0, r1 = 0;
    std::string arena;
    std::vector<AttrSet> sets;       // local first-appearance order
    std::map<AttrSet, uint32_t> ids;
  };
  // ranges of about equal span counts; one range below a few thousand spans
  const int width = N >= 4096 ? std::min<int>(parallel_width(), (int)std::min<size_t>(R, N / 2048)) : 1;
  const int nr = std::max(1, width);
  std::vector<Range> rg((size_t)nr);
  for (int k = 0, ri = 0; k < nr; k++) {
    rg[k].r0 = (size_t)ri;
    const uint64_t goal = N * (uint64_t)(k + 1) / (uint64_t)nr;
    while ((size_t)ri < R && (span0[ri + 1] <= goal || k == nr - 1)) ri++;
    rg[k].r1 = (size_t)ri;
  }
  auto fill = [&](int k) {
    Range& g = rg[(size_t)k];
    ProtoSizer sizer;
    SpanCols sc;
    auto add_str = [&](std::string_view v) {
      ose_strref r{(uint32_t)g.arena.size(), (uint32_t)v.size()};
      g.arena.append(v.data(), v.size());
      return r;
    };
    for (size_t ri = g.r0; ri < g.r1; ri++) {
      const ResourceSpans& rs = t.resource_spans[ri];
      const ResourceCols rc = columnize_resource(ctx_, rs.resource_attrs);
      hb->res_svc[ri] = rc.svc;
      hb->res_svc_str[ri] = rc.svc_str;
      hb->res_url_ok[ri] = rc.url_ok;
      auto it = g.ids.find(rc.attrset);
      if (it == g.ids.end()) {
        it = g.ids.emplace(rc.attrset, (uint32_t)g.sets.size()).first;
        g.sets.push_back(rc.attrset);
      }
      hb->res_attrset[ri] = it->second;   // local id until the merge
      hb->res_size[ri] = (uint32_t)sizer.resource_fixed(rs);
      uint64_t i = span0[ri], sidx = scope0[ri];
      for (auto& ss : rs.scope_spans) {
        hb->scope_size[sidx] = (uint32_t)sizer.scope_fixed(ss);
        hb->scope_resource[sidx] = (uint32_t)ri;
        for (auto& sp : ss.spans) {
          columnize_span(ctx_, sp, rc.attr_res, sizer, sc);
          hb->trace_id[2 * i] = sc.hi;
          hb->trace_id[2 * i + 1] = sc.lo;
          hb->start[i] = sc.start;
          hb->end[i] = sc.end;
          hb->status[i] = sc.status;
          hb->kind[i] = sc.kind;
          hb->resource[i] = (uint32_t)ri;
          hb->scope[i] = (uint32_t)sidx;
          hb->span_size[i] = sc.span_size;
          hb->name_len[i] = sc.name_len;
          for (size_t w = 0; w < W && w < sc.attr_match.size(); w++) hb->attr_match[w * N + i] = sc.attr_match[w];
          for (size_t q = 0; q < nk; q++) {
            uint64_t v = sc.attr_val[q];
            if (sc.attr_type[q] == OSE_ATTR_STR) {
              const ose_strref r = add_str(sc.attr_str[q]);
              v = (uint64_t)r.off | ((uint64_t)r.len << 32);
            }
            hb->attr_type[q * N + i] = sc.attr_type[q];
            hb->attr_val[q * N + i] = v;
          }
          // absent strings: {~0, 0} until the merge makes them {0, 0} (a
          // present empty string keeps its place, as in a sequential walk)
          hb->route[i] = sc.has_route ? add_str(sc.route) : ose_strref{~0u, 0};
          hb->url_flags[i] = sc.url_flags;
          hb->path[i] = (sc.url_flags & OSE_URL_PATH_MASK) != OSE_URL_PATH_NONE ? add_str(sc.path) : ose_strref{~0u, 0};
          i++;
        }
        sidx++;
      }
    }
  };
  if (nr > 1) parallel_run(nr, fill);
  else fill(0);
  // merge: attribute sets in first-appearance order, arenas concatenated
  std::map<AttrSet, uint32_t> gid;
  std::vector<uint64_t> abase((size_t)nr + 1, 0);
  std::vector<std::vector<uint32_t>> remap((size_t)nr);
  for (int k = 0; k < nr; k++) {
    for (auto& set : rg[k].sets) {
      auto it = gid.find(set);
      if (it == gid.end()) {
        it = gid.emplace(set, (uint32_t)hb->attrsets.size()).first;
        hb->attrsets.push_back(set);
      }
      remap[k].push_back(it->second);
    }
    abase[k + 1] = abase[k] + rg[k].arena.size();
  }
  const size_t abytes = abase[nr];
  hb->arena.resize(((abytes + 15) / 16) * 16 + 16, 0);
  auto place = [&](int k) {
    Range& g = rg[(size_t)k];
    if (!g.arena.empty()) std::memcpy(hb->arena.data() + abase[k], g.arena.data(), g.arena.size());
    for (size_t ri = g.r0; ri < g.r1; ri++) hb->res_attrset[ri] = remap[k][hb->res_attrset[ri]];
    const uint32_t base = (uint32_t)abase[k];
    for (uint64_t i = span0[g.r0]; i < span0[g.r1]; i++) {
      ose_strref& rt = hb->route[i];
      rt = rt.off == ~0u ? ose_strref{0, 0} : ose_strref{rt.off + base, rt.len};
      ose_strref& pt = hb->path[i];
      pt = pt.off == ~0u ? ose_strref{0, 0} : ose_strref{pt.off + base, pt.len};
      if (base)
        for (size_t q = 0; q < nk; q++)
          if (hb->attr_type[q * N + i] == OSE_ATTR_STR) hb->attr_val[q * N + i] += base;   // off in the low half
    }
  };
  if (nr > 1) parallel_run(nr, place);
  else place(0);
  const std::string_view arena(reinterpret_cast<const char*>(hb->arena.data()), abytes);
  size_t n = N;
  hb->cols.n_spans = n;
  hb->cols.n_resources = (uint32_t)R;
  hb->cols.n_scopes = (uint32_t)S;
  hb->cols.n_attrsets = (uint32_t)hb->attrsets.size();
  hb->cols.arena_bytes = arena.size();
  hb->cols.n_attr_keys = (uint32_t)nk;
  if (hb->attr_type.empty()) hb->attr_type.push_back(0), hb->attr_val.push_back(0);
  // outputs (vectors never empty so data() is non-null)
  size_t nn = std::max<size_t>(n, 1);
  hb->keep.assign(nn, 0);
  hb->trace_keep.assign(nn, 0);
  hb->trace_level.assign(nn, 0);
  hb->trace_ratio.assign(nn, 0);
  hb->trace_first_span.assign(nn, 0);
  hb->trace_count.assign(1, 0);
  hb->url_out.assign(nn, 0);
  hb->tmpl.assign(nn, ose_strref{0, 0});
  // capacity bound: every output byte comes from a path byte, a separator or
  // a name (the test seam's oracle writes here; ProcessTraces sizes it to
  // what the device used when it reads the outputs back)
  size_t cap = 0;
  if (keep_copy) {
    cap = 16 + arena.size() * 2;
    uint32_t maxname = 5;
    for (auto& c : url_.custom_ids) maxname = std::max<uint32_t>(maxname, (uint32_t)c.template_name.size());
    for (auto& r : url_.templatization_rules) maxname = std::max<uint32_t>(maxname, (uint32_t)r.size());
    for (size_t i = 0; i < n; i++) cap += 2 + (size_t)(hb->path[i].len + 1) * (maxname + 3);
  }
  hb->tmpl_arena.assign(cap + 16, 0);
  hb->attrset_bytes.assign(std::max<size_t>(hb->attrsets.size(), 1), 0);
  hb->accepted.assign(1, 0);
  hb->res_bytes.assign(std::max<size_t>(hb->res_svc.size(), 1), 0);
  hb->tmpl_used.assign(1, 0);
  hb->device_status.assign(4, 0);
  for (auto* v : {&hb->res_svc, &hb->res_svc_str, &hb->res_attrset, &hb->res_size, &hb->scope_size, &hb->scope_resource,
                  &hb->resource, &hb->scope, &hb->span_size, &hb->name_len})
    if (v->empty()) v->push_back(0);
  for (auto* v : {&hb->status, &hb->kind, &hb->url_flags, &hb->res_url_ok})
    if (v->empty()) v->push_back(0);
  for (auto* v : {&hb->trace_id, &hb->start, &hb->end, &hb->attr_match})
    if (v->empty()) v->push_back(0);
  if (hb->path.empty()) hb->path.push_back(ose_strref{0, 0});
  if (hb->route.empty()) hb->route.push_back(ose_strref{0, 0});
  hb->bind();
  return hb;
}

void TracesProcessor::Apply(HostBatch& hb, Traces& td) {
  const uint32_t st = stages();
  const ose_outputs& o = hb.outs;
  // odigossampling: drop the spans of unsampled traces.  With one trace per
  // call (OSE_GROUP_BATCH) this is exactly ResourceSpans().RemoveIf(true)
  // (processor.go:23-25); per trace_id, emptied scopes/resources go too.
  const bool sampled = st & OSE_STAGE_SAMPLE;
  const bool by_trace = sampled && group_mode != OSE_GROUP_BATCH;
  const size_t R = td.resource_spans.size();
  std::vector<uint64_t> span0(R + 1, 0);
  for (size_t ri = 0; ri < R; ri++) {
    uint64_t ns = 0;
    for (auto& ss : td.resource_spans[ri].scope_spans) ns += ss.spans.size();
    span0[ri + 1] = span0[ri] + ns;
  }
  const uint64_t N = span0[R];
  std::vector<uint8_t> drop_res(R, 0);
  // Kept spans and scopes are swapped forward in order (RemoveIf), the
  // dropped ones destroyed by one resize per scope list at the end.
  std::vector<uint64_t> scope0(R + 1, 0);
  for (size_t ri = 0; ri < R; ri++) scope0[ri + 1] = scope0[ri] + td.resource_spans[ri].scope_spans.size();
  std::vector<uint32_t> span_keep(by_trace ? scope0[R] : 0), scope_keep(by_trace ? R : 0);
  // Ranges of resources are applied in parallel on the host task pool for a
  // large batch.  A pool thread frees nothing of the caller's objects: a
  // string or attribute list it replaces is moved to its range's `old` list
  // (new memory comes from the pool thread's own malloc arena), and those,
  // like the dropped spans, are destroyed on the calling thread afterwards —
  // frees from several threads into the caller's arena serialise on its lock
  // (measured on the GPU box: plain in-place mutation took 77 ns/span on one
  // thread and 460 on four).
  struct Old {
    std::vector<std::string> strs;
    std::vector<std::vector<KV>> lists;
  };
  auto put_str = [](Old& old, AttrMap& m, std::string_view k, std::string_view v) {   // pcommon.Map.PutStr
    for (auto& e : m.kv)
      if (e.first == k) {
        if (e.second.type == Value::TStr && v.size() <= e.second.s.capacity()) {
          e.second.s.assign(v.data(), v.size());
        } else {
          Value nv = Value::str(std::string(v));
          std::swap(e.second, nv);
          if (!nv.s.empty() || !nv.map.empty() || !nv.slice.empty()) {
            old.strs.push_back(std::move(nv.s));
            if (!nv.map.empty()) old.lists.push_back(std::move(nv.map));
          }
        }
        return;
      }
    if (m.kv.size() == m.kv.capacity()) {   // grow without freeing the old list here
      std::vector<KV> nkv;
      nkv.reserve(m.kv.size() * 2 + 1);
      for (auto& e : m.kv) nkv.push_back(std::move(e));
      std::swap(m.kv, nkv);
      old.lists.push_back(std::move(nkv));
    }
    m.kv.emplace_back(std::string(k), Value::str(std::string(v)));
  };
  auto apply_range = [&](size_t r0, size_t r1, Old& old) {
    for (size_t ri = r0; ri < r1; ri++) {
      ResourceSpans& rs = td.resource_spans[ri];
      uint64_t i = span0[ri];
      bool had = false;
      uint32_t ws = 0;
      for (size_t si = 0; si < rs.scope_spans.size(); si++) {
        ScopeSpans& ss = rs.scope_spans[si];
        const bool shad = !ss.spans.empty();
        had |= shad;
        size_t w = 0;
        for (size_t q = 0; q < ss.spans.size(); q++, i++) {
          Span& sp = ss.spans[q];
          const bool kept = !sampled || o.keep[i];
          if (kept && (st & OSE_STAGE_TEMPLATE) && o.url_out[i]) {
            const std::string_view tmpl(reinterpret_cast<const char*>(o.tmpl_arena) + o.tmpl[i].off, o.tmpl[i].len);
            if (o.url_out[i] & OSE_OUT_SET_ATTR)   // processor.go:259
              put_str(old, sp.attrs, sp.kind == OSE_KIND_CLIENT ? "url.template" : "http.route", tmpl);
            if (o.url_out[i] & OSE_OUT_RENAME) {
              const Value* m = sp.attrs.Get("http.request.method");
              if (!m) m = sp.attrs.Get("http.method");
              std::string nm = m ? m->AsString() : std::string();   // processor.go:230-232
              nm.reserve(nm.size() + 1 + tmpl.size());
              nm += ' ';
              nm += tmpl;
              std::swap(sp.name, nm);
              old.strs.push_back(std::move(nm));
            }
          }
          if (by_trace && kept) {   // RemoveIf, keeping order
            if (w != q) std::swap(ss.spans[w], sp);
            w++;
          }
        }
        // an emptied scope goes; a scope that never had spans stays
        if (by_trace && (w || !shad)) {
          span_keep[scope0[ri] + ws] = (uint32_t)w;   // by the scope's new place
          if (ws != si) std::swap(rs.scope_spans[ws], ss);
          ws++;
        }
      }
      if (by_trace) {
        scope_keep[ri] = ws;
        if (had && ws == 0) drop_res[ri] = 1;
      }
    }
  };
  const int nr = N >= 4096 ? std::max(1, std::min<int>(parallel_width(), (int)std::min<uint64_t>(R, N / 2048))) : 1;
  std::vector<Old> olds((size_t)nr);
  if (nr > 1) {
    std::vector<size_t> cut((size_t)nr + 1, R);
    cut[0] = 0;
    for (int k = 1, ri = 0; k < nr; k++) {
      const uint64_t goal = N * (uint64_t)k / (uint64_t)nr;
      while ((size_t)ri < R && span0[ri + 1] <= goal) ri++;
      cut[k] = (size_t)ri;
    }
    parallel_run(nr, [&](int k) { apply_range(cut[k], cut[k + 1], olds[(size_t)k]); });
  } else {
    apply_range(0, R, olds[0]);
  }
  olds.clear();
  if (by_trace) {   // the dropped spans and scopes
    for (size_t ri = 0; ri < R; ri++) {
      auto& sv = td.resource_spans[ri].scope_spans;
      sv.resize(scope_keep[ri]);
      for (size_t k = 0; k < sv.size(); k++) sv[k].spans.resize(span_keep[scope0[ri] + k]);
    }
  }
  if (sampled) {
    if (group_mode == OSE_GROUP_BATCH) {
      // one decision for the whole call, spanless resources included
      if (!o.trace_keep[0]) td.resource_spans.clear();
    } else {
      size_t w = 0;
      for (size_t ri = 0; ri < R; ri++) {
        if (drop_res[ri]) continue;
        if (w != ri) td.resource_spans[w] = std::move(td.resource_spans[ri]);
        w++;
      }
      td.resource_spans.resize(w);
    }
  }
  if (st & OSE_STAGE_SIZE) {
    std::lock_guard<std::mutex> g(mu_);
    for (size_t a = 0; a < hb.attrsets.size(); a++)
      if (o.attrset_bytes[a]) data_size_[hb.attrsets[a]] += o.attrset_bytes[a];
    accepted_spans_ += o.accepted_spans[0];
  }
}

int TracesProcessor::ProcessTraces(Traces& td, double* phase_s) {
  using clk = std::chrono::steady_clock;
  auto t0 = clk::now();
  auto lap = [&](int k) {
    if (!phase_s) return;
    auto t = clk::now();
    phase_s[k] += std::chrono::duration<double>(t - t0).count();
    t0 = t;
  };
  ose_rand rnd{0, 0.0};
  int rc;
  {
    std::lock_guard<std::mutex> g(mu_);
    rc = ensure_engine();
    if (rc) return rc;
    rnd.seed = seed_ ^ (draws_ * 0x9E3779B97F4A7C15ull);
    if (has_traffic_) rnd.traffic_u = next_uniform();   // rand.Float64() per call (processor.go:72)
  }
  auto hb = Columnarize(td);
  lap(0);
  ose_columns dims = hb->cols;
  ose_batch* b = nullptr;
  rc = ose_batch_acquire(eng_, &dims, &b);
  if (rc) return rc;
  ose_columns* c = ose_batch_columns(b);
  ose_outputs* o = ose_batch_outputs(b);
  // outputs Apply does not read are not produced (no per-trace compaction,
  // no D2H): one decision per call in BATCH mode, keep bytes otherwise
  o->trace_first_span = nullptr;
  o->trace_level = nullptr;
  o->trace_ratio = nullptr;
  o->res_bytes = nullptr;
  if (group_mode != OSE_GROUP_BATCH) o->trace_count = nullptr, o->trace_keep = nullptr;
  const uint64_t n = hb->cols.n_spans;
  const uint32_t R = hb->cols.n_resources, S = hb->cols.n_scopes, A = hb->cols.n_attrsets;
  auto cp = [](const void* dst, const void* src, size_t bytes) {
    if (bytes) std::memcpy(const_cast<void*>(dst), src, bytes);
  };
  cp(c->arena, hb->cols.arena, hb->cols.arena_bytes);
  cp(c->trace_id, hb->cols.trace_id, 16 * n);
  cp(c->start_ns, hb->cols.start_ns, 8 * n);
  cp(c->end_ns, hb->cols.end_ns, 8 * n);
  cp(c->status, hb->cols.status, n);
  cp(c->kind, hb->cols.kind, n);
  cp(c->resource, hb->cols.resource, 4 * n);
  cp(c->scope, hb->cols.scope, 4 * n);
  cp(c->url_flags, hb->cols.url_flags, n);
  cp(c->path, hb->cols.path, 8 * n);
  cp(c->route, hb->cols.route, 8 * n);
  cp(c->span_size, hb->cols.span_size, 4 * n);
  cp(c->name_len, hb->cols.name_len, 4 * n);
  cp(c->res_svc, hb->cols.res_svc, 4 * R);
  cp(c->res_svc_str, hb->cols.res_svc_str, 4 * R);
  cp(c->res_url_ok, hb->cols.res_url_ok, R);
  cp(c->res_attrset, hb->cols.res_attrset, 4 * R);
  cp(c->res_size, hb->cols.res_size, 4 * R);
  cp(c->scope_size, hb->cols.scope_size, 4 * S);
  cp(c->scope_resource, hb->cols.scope_resource, 4 * S);
  cp(c->attr_match, hb->cols.attr_match, 8 * n * std::max<uint32_t>(1, hb->cols.attr_match_words));
  if (hb->cols.n_attr_keys) {
    cp(c->attr_type, hb->cols.attr_type, (size_t)hb->cols.n_attr_keys * n);
    cp(c->attr_val, hb->cols.attr_val, 8 * (size_t)hb->cols.n_attr_keys * n);
  }
  std::memset(o->attrset_bytes, 0, 8 * (size_t)A);
  std::memset(o->accepted_spans, 0, 8);
  lap(1);
  rc = ose_process(eng_, b, stages(), group_mode, &rnd);
  if (rc) { ose_batch_release(b); return rc; }
  lap(2);
  // read back into the host batch and apply
  cp(hb->outs.keep, o->keep, n);
  if ((stages() & OSE_STAGE_SAMPLE) && group_mode == OSE_GROUP_BATCH) {
    cp(hb->outs.trace_count, o->trace_count, 4);
    cp(hb->outs.trace_keep, o->trace_keep, 1);
  }
  cp(hb->outs.url_out, o->url_out, n);
  cp(hb->outs.tmpl, o->tmpl, 8 * n);
  uint64_t used = *o->tmpl_arena_used;
  if (used + 16 > hb->tmpl_arena.size()) { hb->tmpl_arena.resize(used + 16); hb->bind(); }
  cp(hb->outs.tmpl_arena, o->tmpl_arena, used);
  cp(hb->outs.attrset_bytes, o->attrset_bytes, 8 * (size_t)A);
  cp(hb->outs.accepted_spans, o->accepted_spans, 8);
  ose_batch_release(b);
  lap(3);
  Apply(*hb, td);
  lap(4);
  return 0;
}

std::string TracesProcessor::MetricsJson() const {
  Json root = Json::object();
  Json pts = Json::array();
  for (auto& kv : data_size_) {
    Json p = Json::object();
    Json at = Json::object();
    for (auto& a : kv.first) at.set(a.first, Json::str(a.second));
    p.set("attributes", std::move(at));
    p.set("value", Json::number(std::to_string(kv.second)));
    pts.push(std::move(p));
  }
  root.set("otelcol_odigos_trace_data_size", std::move(pts));
  root.set("otelcol_odigos_accepted_spans", Json::number(std::to_string(accepted_spans_)));
  std::string s;
  dump_json(s, root);
  return s;
}

}  // namespace ose

// ---------------- C API for the host layer (tests, smoke) ----------------
using namespace ose;

namespace {
thread_local std::string g_host_err;
char* dup_cstr(const std::string& s) {
  char* p = static_cast<char*>(std::malloc(s.size() + 1));
  std::memcpy(p, s.data(), s.size());
  p[s.size()] = 0;
  return p;
}
std::string dump_traces(const Traces& t) {
  std::string s;
  dump_json(s, traces_to_json(t));
  return s;
}
}  // namespace

extern "C" {

const char* osehost_last_error(void) { return g_host_err.c_str(); }

// Factory.CreateTraces for "odigossampling" | "odigosurltemplate" |
// "odigostrafficmetrics" | "pipeline" (all three, gateway order).  NULL on a
// config error (message in osehost_last_error).
void* osehost_processor_create(const char* type, const char* cfg_json) {
  ProcKind k;
  std::string t = type ? type : "";
  if (t == "odigossampling") k = ProcKind::Sampling;
  else if (t == "odigosurltemplate") k = ProcKind::UrlTemplate;
  else if (t == "odigostrafficmetrics") k = ProcKind::TrafficMetrics;
  else if (t == "pipeline") k = ProcKind::Pipeline;
  else { g_host_err = "unknown processor type: " + t; return nullptr; }
  Json cfg;
  try {
    cfg = parse_json(cfg_json && *cfg_json ? cfg_json : "{}");
  } catch (const std::exception& e) {
    g_host_err = e.what();
    return nullptr;
  }
  auto* p = new TracesProcessor(k, cfg);
  if (!p->error().empty()) { g_host_err = p->error(); delete p; return nullptr; }
  return p;
}

void osehost_processor_destroy(void* p) { delete static_cast<TracesProcessor*>(p); }

void osehost_processor_set(void* p, uint64_t seed, uint32_t group_mode) {
  auto* tp = static_cast<TracesProcessor*>(p);
  tp->set_seed(seed);
  tp->group_mode = group_mode;
}

// ConsumeTraces on the device path.  Returns 0 and the processed traces as
// OTLP/JSON in *out (free with osehost_free), or an OSE_E* code.
int osehost_consume(void* p, const char* traces_json, char** out) {
  auto* tp = static_cast<TracesProcessor*>(p);
  Traces td;
  try {
    td = traces_from_json(parse_json(traces_json));
  } catch (const std::exception& e) {
    g_host_err = e.what();
    return OSE_EINVAL;
  }
  int rc = tp->ProcessTraces(td);
  if (rc) { g_host_err = ose_last_error(); return rc; }
  if (out) *out = dup_cstr(dump_traces(td));
  return 0;
}

// Test seam: the host half of ConsumeTraces without the device.
void* osehost_columnarize(void* p, const char* traces_json) {
  auto* tp = static_cast<TracesProcessor*>(p);
  try {
    return tp->Columnarize(traces_from_json(parse_json(traces_json)), true).release();   // osehost_apply reads the copy
  } catch (const std::exception& e) {
    g_host_err = e.what();
    return nullptr;
  }
}
ose_columns* osehost_batch_columns(void* hb) { return &static_cast<HostBatch*>(hb)->cols; }
ose_outputs* osehost_batch_outputs(void* hb) { return &static_cast<HostBatch*>(hb)->outs; }
int osehost_apply(void* p, void* hb, char** out) {
  auto* tp = static_cast<TracesProcessor*>(p);
  auto* b = static_cast<HostBatch*>(hb);
  Traces td = b->td;
  tp->Apply(*b, td);
  if (out) *out = dup_cstr(dump_traces(td));
  return 0;
}
void osehost_batch_free(void* hb) { delete static_cast<HostBatch*>(hb); }

// Drop-in timing (tools/dropin_bench.py): ConsumeTraces end to end on the
// C++ host mirror.  traces_json is a JSON array of OTLP/JSON Traces; thread t
// of `threads` consumes items t, t+threads, ... `reps` times each, every call
// on a fresh copy of its item (the copy is outside the timed call).
// out[0] wall s, [1] calls, [2] spans, [3..7] summed phase s (columnarise,
// pinned fill, ose_process, read-back, apply), [8..11] per-call latency
// p50/p90/p99/max s.  Returns 0 or the first failing call's code.
int osehost_bench(void* p, const char* traces_json, uint32_t reps, uint32_t threads, double* out) {
  auto* tp = static_cast<TracesProcessor*>(p);
  std::vector<Traces> items;
  try {
    Json arr = parse_json(traces_json);
    if (!arr.is_arr()) throw std::runtime_error("expected a JSON array of Traces");
    for (auto& t : arr.arr) items.push_back(traces_from_json(t));
  } catch (const std::exception& e) {
    g_host_err = e.what();
    return OSE_EINVAL;
  }
  if (threads < 1) threads = 1;
  std::vector<std::vector<double>> lat(threads);
  std::vector<std::array<double, 5>> ph(threads);
  std::atomic<int> first_rc{0};
  std::string first_err;
  std::mutex err_mu;
  uint64_t spans = 0;
  for (auto& t : items)
    for (auto& rs : t.resource_spans)
      for (auto& ss : rs.scope_spans) spans += ss.spans.size();
  using clk = std::chrono::steady_clock;
  // every call's Traces is copied before the clock starts (by the thread that
  // makes the call, as a receiver allocates the pdata it hands on) and
  // destroyed after it stops: the copy and the teardown are the caller's.
  // The copies held at once are bounded (about 1M spans per thread): reps
  // beyond that are dropped, and out[1] / out[2] count the calls made.
  {
    const uint64_t per_rep = std::max<uint64_t>(1, (spans + threads - 1) / threads);
    const uint64_t budget = 1ull << 20;
    reps = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(reps, budget / per_rep));
  }
  std::vector<std::vector<Traces>> work(threads);
  std::atomic<uint32_t> ready{0};
  std::atomic<bool> go{false};
  clk::time_point t0;
  std::vector<std::thread> th;
  for (uint32_t w = 0; w < threads; w++)
    th.emplace_back([&, w]() {
      ph[w].fill(0.0);
      for (uint32_t r = 0; r < reps; r++)
        for (size_t i = w; i < items.size(); i += threads) work[w].push_back(items[i]);
      if (ready.fetch_add(1) + 1 == threads) {
        t0 = clk::now();
        go.store(true, std::memory_order_release);
      }
      while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
      size_t next = 0;
      for (uint32_t r = 0; r < reps; r++)
        for (size_t i = w; i < items.size(); i += threads) {
          Traces& td = work[w][next++];
          auto a = clk::now();
          int rc = tp->ProcessTraces(td, ph[w].data());
          lat[w].push_back(std::chrono::duration<double>(clk::now() - a).count());
          if (rc) {
            int z = 0;
            if (first_rc.compare_exchange_strong(z, rc)) {
              std::lock_guard<std::mutex> g(err_mu);
              first_err = ose_last_error();   // thread-local in the worker
            }
            return;
          }
        }
    });
  for (auto& x : th) x.join();
  const double wall = std::chrono::duration<double>(clk::now() - t0).count();
  std::vector<double> all;
  for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
  std::sort(all.begin(), all.end());
  auto pct = [&](double q) { return all.empty() ? 0.0 : all[std::min(all.size() - 1, (size_t)(q * (double)all.size()))]; };
  out[0] = wall;
  out[1] = (double)all.size();
  out[2] = (double)spans * reps;
  for (int k = 0; k < 5; k++) {
    out[3 + k] = 0;
    for (auto& v : ph) out[3 + k] += v[k];
  }
  out[8] = pct(0.50);
  out[9] = pct(0.90);
  out[10] = pct(0.99);
  out[11] = all.empty() ? 0.0 : all.back();
  if (first_rc.load()) { g_host_err = first_err; return first_rc.load(); }
  return 0;
}

char* osehost_metrics_json(void* p) { return dup_cstr(static_cast<TracesProcessor*>(p)->MetricsJson()); }
// OTLP protobuf -> pdata (otlp_pb.cpp) -> OTLP/JSON: the host unmarshaler
// the ingest's host pass uses (tests); NULL + osehost_last_error on error
char* osehost_pb_to_json(const uint8_t* pb, size_t len) {
  Traces td;
  std::string err;
  if (!traces_from_protobuf(pb, len, td, err)) {
    g_host_err = err;
    return nullptr;
  }
  return dup_cstr(dump_traces(td));
}
// Traces round trip through the pdata model (fixture sanity)
char* osehost_roundtrip(const char* traces_json) {
  try {
    return dup_cstr(dump_traces(traces_from_json(parse_json(traces_json))));
  } catch (const std::exception& e) {
    g_host_err = e.what();
    return nullptr;
  }
}
// ptrace.ProtoMarshaler.ResourceSpansSize for every resource of a batch
int osehost_resource_sizes(const char* traces_json, int gogo, uint64_t* out, size_t cap) {
  try {
    Traces t = traces_from_json(parse_json(traces_json));
    ProtoSizer s;
    s.gogo = gogo != 0;
    for (size_t k = 0; k < t.resource_spans.size() && k < cap; k++) out[k] = s.resource_spans(t.resource_spans[k]);
    return (int)t.resource_spans.size();
  } catch (const std::exception& e) {
    g_host_err = e.what();
    return -1;
  }
}
char* osehost_as_string(const char* value_json) {   // pcommon.Value.AsString of an OTLP/JSON AnyValue
  try {
    Json j = parse_json(value_json);
    Json wrapper = Json::object();
    Json attrs = Json::array();
    Json kv = Json::object();
    kv.set("key", Json::str("k"));
    kv.set("value", j);
    attrs.push(kv);
    Json res = Json::object();
    res.set("attributes", attrs);
    Json rs = Json::object();
    rs.set("resource", res);
    Json rss = Json::array();
    rss.push(rs);
    wrapper.set("resourceSpans", rss);
    Traces t = traces_from_json(wrapper);
    return dup_cstr(t.resource_spans[0].resource_attrs.kv[0].second.AsString());
  } catch (const std::exception& e) {
    g_host_err = e.what();
    return nullptr;
  }
}
void osehost_free(char* s) { std::free(s); }

}  // extern "C"

// ---- test seam: the product regex->DFA compiler evaluated on the host ----
#include "regex_dfa.hpp"
// One span_attribute condition on one attribute value (tests): rule_json is
// the rule_details object, value_json an OTLP/JSON AnyValue.  1 / 0, or -1
// with osehost_last_error() when the rule cannot be compiled.
extern "C" int osehost_span_attr_eval(const char* rule_json, const char* value_json) {
  try {
    ose::Json d = ose::parse_json(rule_json);
    ose::SpanAttributeRule r;
    auto gs = [&](const char* k, std::string& out) {
      if (const ose::Json* v = d.get(k)) out = v->s;
    };
    gs("service_name", r.service_name);
    gs("attribute_key", r.attribute_key);
    gs("condition_type", r.condition_type);
    gs("operation", r.operation);
    gs("expected_value", r.expected_value);
    gs("json_path", r.json_path);
    ose::SpanAttrPredicate p;
    std::string e = p.compile(r);
    if (!e.empty()) { g_host_err = e; return -1; }
    ose::Json vj = ose::parse_json(value_json);
    ose::Json wrapper = ose::Json::object();
    ose::Json attrs = ose::Json::array();
    ose::Json kv = ose::Json::object();
    kv.set("key", ose::Json::str("k"));
    kv.set("value", vj);
    attrs.push(kv);
    ose::Json res = ose::Json::object();
    res.set("attributes", attrs);
    ose::Json rs = ose::Json::object();
    rs.set("resource", res);
    ose::Json rss = ose::Json::array();
    rss.push(rs);
    wrapper.set("resourceSpans", rss);
    ose::Traces t = ose::traces_from_json(wrapper);
    return p.eval(t.resource_spans[0].resource_attrs.kv[0].second) ? 1 : 0;
  } catch (const std::exception& ex) {
    g_host_err = ex.what();
    return -1;
  }
}

extern "C" int osehost_regex_match(const char* pattern, const char* s, size_t n) {
  ose::Dfa d;
  std::string err;
  ose::RegexStatus st = ose::compile_dfa(pattern, d, err);
  if (st == ose::RegexStatus::Syntax) { g_host_err = err; return -1; }
  if (st != ose::RegexStatus::Ok) { g_host_err = err; return -2; }
  return ose::dfa_match(d, reinterpret_cast<const uint8_t*>(s), n) ? 1 : 0;
}

// The host matcher (HostRegexp) with the given full-DFA caps; *lazy = 1 when
// the pattern went to the lazy DFA.  1 / 0, -1 syntax, -2 unsupported.
extern "C" int osehost_regex_match_host(const char* pattern, const char* s, size_t n, uint32_t max_states,
                                        uint64_t max_bytes, int* lazy) {
  ose::HostRegexp re;
  std::string err;
  ose::RegexStatus st = re.compile(pattern, err, max_states, max_bytes);
  if (st == ose::RegexStatus::Syntax) { g_host_err = err; return -1; }
  if (st != ose::RegexStatus::Ok) { g_host_err = err; return -2; }
  if (lazy) *lazy = re.lazy() ? 1 : 0;
  return re.match(reinterpret_cast<const uint8_t*>(s), n) ? 1 : 0;
}
