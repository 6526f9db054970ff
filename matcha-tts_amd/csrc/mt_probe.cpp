#include "mt_probe.h"
#include "mt_vconv.h"

#include <algorithm>
#include <mutex>
#include <vector>

namespace mt {
namespace {
std::mutex g_mu;
int g_site = PROBE_NONE;
std::vector<hipEvent_t> g_ev;  // 2 per launch: begin, end
int g_n = 0, g_cap = 0;
double g_flops = 0, g_bytes = 0;
std::vector<double> g_lf, g_lb;  // per launch: algorithmic FLOPs, bytes
std::vector<int> g_lt;           // per launch: kernel tag
bool g_open = false;
bool g_paused = false;

void release() {
  for (hipEvent_t e : g_ev) (void)hipEventDestroy(e);
  g_ev.clear();
  g_n = g_cap = 0;
  g_flops = g_bytes = 0;
  g_lf.clear();
  g_lb.clear();
  g_lt.clear();
  g_site = PROBE_NONE;
  g_open = false;
  g_paused = false;
}
}  // namespace

bool probe_armed(int site) { return g_site != PROBE_NONE && g_site == site; }
bool probe_any_armed() { return g_site != PROBE_NONE; }

void probe_begin(int site, hipStream_t st) {
  if (!probe_armed(site)) return;
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_n >= g_cap || g_open || g_paused) return;
  (void)hipEventRecord(g_ev[2 * g_n], st);
  g_open = true;
}

void probe_end(int site, hipStream_t st, double flops, double bytes, int tag) {
  if (!probe_armed(site)) return;
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_open) return;
  (void)hipEventRecord(g_ev[2 * g_n + 1], st);
  g_open = false;
  ++g_n;
  g_flops += flops;
  g_bytes += bytes;
  g_lf.push_back(flops);
  g_lb.push_back(bytes);
  g_lt.push_back(tag);
}

int probe_detail(int cap, double* ms, double* flops, double* bytes, int* tags) {
  std::lock_guard<std::mutex> lk(g_mu);
  const int n = std::min(cap, g_n);
  for (int i = 0; i < n; ++i) {
    float t = 0.f;
    if (hipEventSynchronize(g_ev[2 * i + 1]) != hipSuccess ||
        hipEventElapsedTime(&t, g_ev[2 * i], g_ev[2 * i + 1]) != hipSuccess) {
      set_error("probe: event timing failed");
      return -1;
    }
    if (ms) ms[i] = t;
    if (flops) flops[i] = g_lf[i];
    if (bytes) bytes[i] = g_lb[i];
    if (tags) tags[i] = g_lt[i];
  }
  return n;
}

int probe_start(int site, int max_launches) {
  std::lock_guard<std::mutex> lk(g_mu);
  release();
  MT_REQUIRE(site > PROBE_NONE && site <= PROBE_VCONV_DEC, "probe: unknown site %d", site);
  MT_REQUIRE(max_launches > 0 && max_launches <= (1 << 16), "probe: max_launches %d", max_launches);
  g_ev.resize(2 * (size_t)max_launches);
  for (hipEvent_t& e : g_ev) MT_CHECK_HIP(hipEventCreate(&e));
  g_cap = max_launches;
  g_site = site;
  return 0;
}

int probe_pause(bool paused) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_paused = paused;
  return 0;
}

int probe_stop(int* launches, double* total_ms, double* flops, double* bytes, double peak_flops, double peak_bw,
               double* roof_ms) {
  std::lock_guard<std::mutex> lk(g_mu);
  double ms = 0, roof = 0;
  for (int i = 0; i < g_n; ++i)  // per-launch roofline time max(F / peak_F, B / peak_BW)
    roof += 1e3 * std::max(peak_flops > 0 ? g_lf[i] / peak_flops : 0.0, peak_bw > 0 ? g_lb[i] / peak_bw : 0.0);
  int rc = 0;
  for (int i = 0; i < g_n && rc == 0; ++i) {
    float t = 0.f;
    if (hipEventSynchronize(g_ev[2 * i + 1]) != hipSuccess ||
        hipEventElapsedTime(&t, g_ev[2 * i], g_ev[2 * i + 1]) != hipSuccess) {
      set_error("probe: event timing failed");
      rc = -1;
    }
    ms += t;
  }
  if (launches) *launches = g_n;
  if (total_ms) *total_ms = ms;
  if (flops) *flops = g_flops;
  if (bytes) *bytes = g_bytes;
  if (roof_ms) *roof_ms = roof;
  release();
  return rc;
}

namespace {
std::vector<int> g_log;
int g_log_cap = 0;
bool g_log_on = false;
}  // namespace

namespace {
struct SchedEntry {
  int rec[SCHED_FIELDS];
  SchedWaits waits;
};
std::vector<SchedEntry>& sched_table() {  // constructed on first use: registrars run during static initialisation
  static std::vector<SchedEntry> t;
  return t;
}
}  // namespace

int sched_register(const int (&rec)[SCHED_FIELDS], SchedWaits waits) {
  auto& t = sched_table();
  for (const auto& e : t)
    if (std::equal(e.rec, e.rec + SCHED_FIELDS, rec)) return 0;
  SchedEntry e;
  std::copy(rec, rec + SCHED_FIELDS, e.rec);
  e.waits = waits;
  t.push_back(e);
  return 0;
}
int sched_count() { return (int)sched_table().size(); }
int sched_get(int i, int* rec, int* wait, int* wait_first, int cap) {
  auto& t = sched_table();
  if (i < 0 || i >= (int)t.size()) return -1;
  std::copy(t[i].rec, t[i].rec + SCHED_FIELDS, rec);
  return t[i].waits(wait, wait_first, cap);
}

void vclog_record(const int (&rec)[VCLOG_FIELDS]) {
  if (!g_log_on) return;
  std::lock_guard<std::mutex> lk(g_mu);
  if ((int)g_log.size() >= g_log_cap * VCLOG_FIELDS) return;
  g_log.insert(g_log.end(), rec, rec + VCLOG_FIELDS);
}

int vclog_start(int cap) {
  std::lock_guard<std::mutex> lk(g_mu);
  MT_REQUIRE(cap > 0 && cap <= (1 << 20), "vconv log: capacity %d", cap);
  g_log.clear();
  g_log.reserve((size_t)cap * VCLOG_FIELDS);
  g_log_cap = cap;
  g_log_on = true;
  return 0;
}

bool vclog_armed() { return g_log_on; }

int vclog_stop(int* out, int cap) {
  std::lock_guard<std::mutex> lk(g_mu);
  const int n = std::min<int>((int)g_log.size() / VCLOG_FIELDS, cap);
  if (out)
    for (int i = 0; i < n * VCLOG_FIELDS; ++i) out[i] = g_log[i];
  g_log.clear();
  g_log_on = false;
  return n;
}

}  // namespace mt
