// size_host.cpp — odigostrafficmetrics: the launch sequence of the size
// stage (size_kernel.hip).
#include <algorithm>

#include "engine_internal.hpp"
#include "kernels.hpp"

namespace ose {

#define HIP_TRY(expr)                                                                                  \
  do {                                                                                                 \
    hipError_t _e = (expr);                                                                            \
    if (_e != hipSuccess) return fail(OSE_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

namespace {
size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
}  // namespace

// [256 | scope sums 8·S | window parts 32·W | window fix flags 4·W | kept
// partials 4·kUrlCopyMaxBlocks | 256], W = the 64-scope windows
namespace {
struct SizeLayout {
  size_t scope, parts, fix, partials, end;
};
SizeLayout size_layout(uint64_t n_scopes) {
  const uint64_t W = (std::max<uint64_t>(n_scopes, 1) + 63) / 64;
  SizeLayout L;
  L.scope = 256;
  L.parts = align_up(L.scope + 8 * std::max<uint64_t>(n_scopes, 1), 256);
  L.fix = align_up(L.parts + 32 * W, 256);
  L.partials = align_up(L.fix + 4 * W, 256);
  L.end = align_up(L.partials + 4ull * kUrlCopyMaxBlocks, 256) + 256;
  return L;
}
}  // namespace
size_t size_scratch_bytes(uint64_t n_scopes, uint64_t n_resources) {
  (void)n_resources;   // the resources are finished in the scopes pass (no per-resource words)
  return size_layout(n_scopes).end;
}

// dataSizesMetricsProcessor.processTraces (odigostrafficmetrics/
// processor.go:71-84) after the stages of `mask` that ran before it in this
// call (gateway order: sampling, then templating, then size): validation, the
// rand gate, the zeroed per-scope / per-resource sums (the workspace from
// byte `off`; the SAMPLE stage's words at its byte 0 hold the OSE_GROUP_BATCH
// decision) and the arguments.  *active is false when the gate skips the
// stage.
int prepare_size(Engine* e, const ose_columns* c, const ose_outputs* o, uint32_t mask, uint32_t group_mode,
                 const ose_rand* rnd, hipStream_t st, Workspace* ws, size_t off, SizeKernelArgs& a, bool& active) {
  active = false;
  if (!e->has_traffic) return fail(OSE_EINVAL, "odigostrafficmetrics is not configured on this engine");
  if (!o->attrset_bytes || !o->accepted_spans) return fail(OSE_EINVAL, "SIZE stage needs attrset_bytes and accepted_spans");
  const uint64_t n = c->n_spans;
  if (n && (!c->span_size || !c->scope)) return fail(OSE_EINVAL, "SIZE stage needs span_size and scope");
  if (c->n_scopes && (!c->scope_size || !c->scope_resource)) return fail(OSE_EINVAL, "SIZE stage needs scope_size and scope_resource");
  if (c->n_resources && (!c->res_size || !c->res_attrset)) return fail(OSE_EINVAL, "SIZE stage needs res_size and res_attrset");
  const bool applied = mask & OSE_STAGE_APPLY_KEEP;   // decisions made by an earlier call
  const bool sampled = (mask & OSE_STAGE_SAMPLE) || applied;
  const bool templated = mask & (OSE_STAGE_TEMPLATE | OSE_STAGE_APPLY_TEMPLATE);   // in this call or an earlier one
  if (applied && n && !o->keep) return fail(OSE_EINVAL, "OSE_STAGE_APPLY_KEEP needs keep");
  if (templated && n && (!c->kind || !c->name_len || !o->url_out || !o->tmpl))
    return fail(OSE_EINVAL, "SIZE after TEMPLATE needs kind, name_len, url_out and tmpl");
  // if p.samplingFraction != 0 && rand.Float64() < p.samplingFraction (processor.go:72)
  const double ratio = e->traffic.sampling_ratio;
  const double u = rnd ? rnd->traffic_u : 0.0;
  if (!(ratio != 0 && u < ratio)) return 0;
  // res_bytes needs no clearing: size_tail_kernel / size_fix_kernel write
  // every entry, zeros when the batch was dropped; the window parts and flags
  // are written every call
  const uint64_t S = c->n_scopes, R = c->n_resources;
  int rc = ws->reserve(off + size_scratch_bytes(S, R));
  if (rc) return rc;
  uint8_t* base = static_cast<uint8_t*>(ws->dev) + off;
  const SizeLayout L = size_layout(S);
  uint8_t* sc = base + L.scope;
  HIP_TRY(hipMemsetAsync(sc, 0, 8 * std::max<uint64_t>(S, 1), st));   // scope sums
  a = SizeKernelArgs{};
  a.n_spans = n;
  a.n_scopes = (uint32_t)S;
  a.n_resources = (uint32_t)R;
  a.n_attrsets = c->n_attrsets;
  a.sampled = sampled;
  a.templated = templated;
  a.remove_empty = applied || (sampled && group_mode == OSE_GROUP_TRACE_ID);
  a.batch_keep = !applied && sampled && group_mode == OSE_GROUP_BATCH
                     ? reinterpret_cast<const uint32_t*>(ws->dev) + kBatchKeepWord : nullptr;
  a.span_size = c->span_size;
  a.name_len = c->name_len;
  a.scope = c->scope;
  a.scope_size = c->scope_size;
  a.scope_resource = c->scope_resource;
  a.res_size = c->res_size;
  a.res_attrset = c->res_attrset;
  a.keep = o->keep;
  a.url_out = o->url_out;
  a.kind = c->kind;
  a.tmpl = o->tmpl;
  a.inverse = e->inverse;
  a.scope_body = reinterpret_cast<uint64_t*>(sc);
  a.parts = reinterpret_cast<SizePart*>(base + L.parts);
  a.fix = reinterpret_cast<uint32_t*>(base + L.fix);
  a.n_swin = (uint32_t)((S + 63) / 64);
  a.attrset_bytes = o->attrset_bytes;
  a.accepted = o->accepted_spans;
  a.res_bytes = o->res_bytes;
  a.kept_partials = nullptr;   // set by run_stages when url_copy_kernel runs the spans pass (size_partials_of)
  a.n_kept_partials = 0;
  active = true;
  return 0;
}

uint32_t* size_partials_of(Workspace* ws, size_t off, uint64_t n_scopes, uint64_t n_resources) {
  (void)n_resources;
  return reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(ws->dev) + off + size_layout(n_scopes).partials);
}

// the spans pass (unless url_copy_kernel ran it: a.kept_partials set), then
// scopes and resources
int run_size_tail(Engine* e, const SizeKernelArgs& a, hipStream_t st) {
  Engine::Timed tm{};
  if (!a.kept_partials) {
    e->prof_begin("size_span_kernel", st, tm);
    launch_size_spans(a, st);
    HIP_TRY(hipGetLastError());
    e->prof_end(tm, st);
  }
  e->prof_begin("size_tail_kernel", st, tm);
  launch_size_tail(a, st);
  HIP_TRY(hipGetLastError());
  e->prof_end(tm, st);
  e->prof_begin("size_fix_kernel", st, tm);
  launch_size_fix(a, st);
  HIP_TRY(hipGetLastError());
  e->prof_end(tm, st);
  return 0;
}

int run_size(Engine* e, const ose_columns* c, const ose_outputs* o, uint32_t mask, uint32_t group_mode,
             const ose_rand* rnd, hipStream_t st, Workspace* ws, size_t off) {
  SizeKernelArgs a;
  bool active = false;
  int rc = prepare_size(e, c, o, mask, group_mode, rnd, st, ws, off, a, active);
  if (rc || !active) return rc;
  return run_size_tail(e, a, st);
}

}  // namespace ose
