#include "profiling.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstring>
#include <condition_variable>
#include <deque>
#include <fstream>
#include <map>
#include <thread>
#include <set>
#include <sstream>

#include "../comm/comm.hpp"
#include "../device/device.hpp"

namespace parsec {

// ============================================================= profiling
namespace {
struct SpillJob {
  ProfilingStream* s;
  std::vector<ProfEvent> events;
  std::vector<uint8_t> info;
};
struct ProfState {
  std::mutex m;
  bool enabled = false;
  std::string filename;
  int rank = 0;
  uint64_t t0 = 0;
  size_t buffer_events = 65536;
  std::vector<DictEntry> dict;
  std::map<std::string, int> dict_index;
  std::vector<ProfilingStream*> streams;
  std::vector<std::pair<std::string, std::string>> infos;
  // writer thread
  std::mutex wm;
  std::condition_variable wcv;
  std::deque<SpillJob> jobs;
  std::thread writer;
  bool writer_stop = false;
  size_t jobs_pending = 0;
  std::condition_variable wdone;
  std::atomic<bool> recording{true};  // parsec_profiling_enable / disable
  std::string last_error;
};
ProfState& P() { static ProfState* s = new ProfState(); return *s; }

void append_file(const std::string& path, const void* data, size_t n) {
  if (!n) return;
  FILE* f = std::fopen(path.c_str(), "ab");
  if (!f) { warning("profiling: cannot append to %s", path.c_str()); return; }
  std::fwrite(data, 1, n, f);
  std::fclose(f);
}

void writer_main() {
  auto& p = P();
  for (;;) {
    SpillJob j;
    {
      std::unique_lock<std::mutex> lk(p.wm);
      p.wcv.wait(lk, [&] { return p.writer_stop || !p.jobs.empty(); });
      if (p.jobs.empty()) return;
      j = std::move(p.jobs.front());
      p.jobs.pop_front();
    }
    append_file(j.s->spill_ev, j.events.data(), j.events.size() * sizeof(ProfEvent));
    append_file(j.s->spill_info, j.info.data(), j.info.size());
    {
      std::lock_guard<std::mutex> lk(p.wm);
      --p.jobs_pending;
    }
    p.wdone.notify_all();
  }
}

// hand the full buffer of `s` to the writer (caller owns s: its thread or lock)
void spill(ProfilingStream* s) {
  auto& p = P();
  SpillJob j;
  j.s = s;
  j.events.swap(s->events);
  j.info.swap(s->info);
  s->spilled_events += j.events.size();
  s->info_base += j.info.size();
  s->events.reserve(p.buffer_events);
  {
    std::lock_guard<std::mutex> lk(p.wm);
    if (!p.writer.joinable()) p.writer = std::thread(writer_main);
    p.jobs.push_back(std::move(j));
    ++p.jobs_pending;
  }
  p.wcv.notify_one();
}

void writer_drain() {
  auto& p = P();
  std::unique_lock<std::mutex> lk(p.wm);
  p.wdone.wait(lk, [&] { return p.jobs_pending == 0; });
}

std::vector<uint8_t> read_all(const std::string& path) {
  std::vector<uint8_t> out;
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return out;
  std::fseek(f, 0, SEEK_END);
  long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  out.resize(n > 0 ? (size_t)n : 0);
  if (n > 0 && std::fread(out.data(), 1, (size_t)n, f) != (size_t)n) out.clear();
  std::fclose(f);
  return out;
}
}  // namespace

bool profiling_enabled() { return P().enabled; }
uint64_t profiling_now() { return now_ns() - P().t0; }

void profiling_init(Context* ctx) {
  auto& p = P();
  std::string fn = ParamRegistry::instance().reg_string("profile", "", "filename", "Write a trace to <filename>-<rank>.prof", "");
  const int64_t be = ParamRegistry::instance().reg_int("profile", "", "buffer_events",
      "Events buffered per stream before the writer thread spills them to disk", 65536);
  std::lock_guard<std::mutex> g(p.m);
  p.buffer_events = (size_t)std::max<int64_t>(be, 16);
  p.rank = ctx->my_rank;
  if (p.t0 == 0) p.t0 = now_ns();
  if (!fn.empty()) { p.enabled = true; p.filename = fn; }
}

void profiling_start() { P().t0 = now_ns(); }

ProfilingStream* profiling_stream_create(const std::string& name) {
  auto* s = new ProfilingStream();
  s->name = name;
  auto& p = P();
  std::lock_guard<std::mutex> g(p.m);
  s->events.reserve(std::min<size_t>(p.buffer_events, 4096));
  s->thread_id = (int)p.streams.size();
  const std::string base = (p.filename.empty() ? std::string("parsec_prof") : p.filename) + "-pid" + std::to_string((long)getpid()) + ".s" + std::to_string(s->thread_id);
  s->spill_ev = base + ".ev.tmp";
  s->spill_info = base + ".info.tmp";
  std::remove(s->spill_ev.c_str());
  std::remove(s->spill_info.c_str());
  p.streams.push_back(s);
  return s;
}

void profiling_thread_init(ExecutionStream* es) {
  if (!P().enabled || es->prof) return;
  es->prof = profiling_stream_create((es->is_manager ? "manager " : "thread ") + std::to_string(es->th_id));
}

void profiling_thread_fini(ExecutionStream* es) { (void)es; }

int profiling_add_dictionary_keyword(const std::string& name, const std::string& attributes, size_t info_length, const std::string& info_desc, int* bkey, int* ekey) {
  auto& p = P();
  std::lock_guard<std::mutex> g(p.m);
  auto it = p.dict_index.find(name);
  int id;
  if (it != p.dict_index.end()) id = it->second;
  else {
    id = (int)p.dict.size();
    p.dict.push_back(DictEntry{name, attributes, info_desc, info_length});
    p.dict_index[name] = id;
  }
  if (bkey) *bkey = 2 * id;
  if (ekey) *ekey = 2 * id + 1;
  return 0;
}

static void trace_into(ProfilingStream* s, int key, uint64_t event_id, uint32_t taskpool_id, uint64_t ts, const void* info, size_t info_len) {
  if (!P().recording.load(std::memory_order_relaxed)) return;
  ProfEvent e;
  e.key = (uint16_t)key;
  e.flags = info_len ? 1 : 0;
  e.taskpool_id = taskpool_id;
  e.event_id = event_id;
  e.timestamp = ts;
  e.info_off = (uint32_t)(s->info_base + s->info.size());
  e.info_len = (uint32_t)info_len;
  if (info_len) s->info.insert(s->info.end(), (const uint8_t*)info, (const uint8_t*)info + info_len);
  s->events.push_back(e);
  if (s->events.size() >= P().buffer_events) spill(s);
}

int profiling_trace(ProfilingStream* s, int key, uint64_t event_id, uint32_t taskpool_id, const void* info, size_t info_len) {
  if (!s) return -1;
  trace_into(s, key, event_id, taskpool_id, profiling_now(), info, info_len);
  return 0;
}

int profiling_trace_at(ProfilingStream* s, int key, uint64_t event_id, uint32_t taskpool_id, uint64_t timestamp, const void* info, size_t info_len) {
  if (!s) return -1;
  std::lock_guard<SpinLock> g(s->lock);
  trace_into(s, key, event_id, taskpool_id, timestamp, info, info_len);
  return 0;
}

std::vector<std::pair<std::string, double>> profiling_rusage() {
  std::vector<std::pair<std::string, double>> out;
  struct rusage ru {};
  if (getrusage(RUSAGE_SELF, &ru) != 0) return out;
  out.emplace_back("ru_utime_s", ru.ru_utime.tv_sec + ru.ru_utime.tv_usec * 1e-6);
  out.emplace_back("ru_stime_s", ru.ru_stime.tv_sec + ru.ru_stime.tv_usec * 1e-6);
  out.emplace_back("ru_maxrss_kb", (double)ru.ru_maxrss);
  out.emplace_back("ru_minflt", (double)ru.ru_minflt);
  out.emplace_back("ru_majflt", (double)ru.ru_majflt);
  out.emplace_back("ru_nvcsw", (double)ru.ru_nvcsw);
  out.emplace_back("ru_nivcsw", (double)ru.ru_nivcsw);
  out.emplace_back("ru_inblock", (double)ru.ru_inblock);
  out.emplace_back("ru_oublock", (double)ru.ru_oublock);
  return out;
}

void profiling_add_information(const std::string& key, const std::string& value) {
  auto& p = P();
  std::lock_guard<std::mutex> g(p.m);
  p.infos.emplace_back(key, value);
}

static void wstr(std::ofstream& o, const std::string& s) {
  uint32_t l = (uint32_t)s.size();
  o.write((const char*)&l, 4);
  o.write(s.data(), l);
}

// Drop every event recorded so far and restart the clock (reference
// parsec_profiling_reset, profiling.c): waits for pending spills, truncates
// the spill files, clears the in-memory tails. Keys and streams are kept.
int profiling_reset() {
  auto& p = P();
  {
    std::unique_lock<std::mutex> lk(p.wm);
    p.wdone.wait(lk, [&] { return p.jobs_pending == 0; });
  }
  std::lock_guard<std::mutex> g(p.m);
  for (auto* s : p.streams) {
    std::lock_guard<SpinLock> sg(s->lock);
    s->events.clear();
    s->info.clear();
    s->info_base = 0;
    s->spilled_events = 0;
    std::remove(s->spill_ev.c_str());
    std::remove(s->spill_info.c_str());
  }
  p.t0 = now_ns();
  return 0;
}

int profiling_dump(const std::string& filename) {
  auto& p = P();
  std::lock_guard<std::mutex> g(p.m);
  std::ofstream o(filename, std::ios::binary);
  if (!o) return -1;
  o.write("PAMDPRF2", 8);
  uint32_t hdr[4] = {(uint32_t)p.rank, (uint32_t)p.dict.size(), (uint32_t)p.streams.size(), (uint32_t)p.infos.size()};
  o.write((const char*)hdr, sizeof(hdr));
  o.write((const char*)&p.t0, 8);
  for (auto& kv : p.infos) { wstr(o, kv.first); wstr(o, kv.second); }
  for (auto& d : p.dict) {
    wstr(o, d.name); wstr(o, d.attributes); wstr(o, d.info_desc);
    uint64_t il = d.info_length;
    o.write((const char*)&il, 8);
  }
  for (auto* s : p.streams) {
    wstr(o, s->name);
    int32_t tid = s->thread_id;
    o.write((const char*)&tid, 4);
    uint32_t ninfo = (uint32_t)s->infos.size();
    o.write((const char*)&ninfo, 4);
    for (auto& kv : s->infos) { wstr(o, kv.first); wstr(o, kv.second); }
    // spilled chunks (in order) + the in-memory tail
    std::vector<uint8_t> sev = read_all(s->spill_ev), sinfo = read_all(s->spill_info);
    uint64_t n = sev.size() / sizeof(ProfEvent) + s->events.size();
    o.write((const char*)&n, 8);
    static_assert(sizeof(ProfEvent) == 32, "event layout");
    o.write((const char*)sev.data(), sev.size());
    o.write((const char*)s->events.data(), s->events.size() * sizeof(ProfEvent));
    uint64_t isz = sinfo.size() + s->info.size();
    o.write((const char*)&isz, 8);
    o.write((const char*)sinfo.data(), sinfo.size());
    o.write((const char*)s->info.data(), s->info.size());
  }
  return o ? 0 : -1;
}

// ---------------------------------------------------- standalone interface
int profiling_standalone_init(int rank) {
  auto& p = P();
  std::lock_guard<std::mutex> g(p.m);
  p.rank = rank;
  if (p.t0 == 0) p.t0 = now_ns();
  return 0;
}

int profiling_dbp_start(const std::string& basefile, const std::string& hr_id) {
  auto& p = P();
  if (basefile.empty()) {
    p.last_error = "dbp_start: empty base file name";
    return -1;
  }
  std::lock_guard<std::mutex> g(p.m);
  p.filename = basefile;
  p.enabled = true;
  p.infos.emplace_back("hr_id", hr_id);
  return 0;
}

int profiling_dbp_dump() {
  auto& p = P();
  writer_drain();
  if (!p.enabled || p.filename.empty()) {
    p.last_error = "dbp_dump: no dbp_start";
    return -1;
  }
  const std::string fn = p.filename + "-" + std::to_string(p.rank) + ".prof";
  if (profiling_dump(fn) != 0) {
    p.last_error = "dbp_dump: cannot write " + fn;
    return -1;
  }
  return 0;
}

int profiling_standalone_fini() {
  auto& p = P();
  writer_drain();
  {
    std::lock_guard<std::mutex> lk(p.wm);
    p.writer_stop = true;
  }
  p.wcv.notify_all();
  if (p.writer.joinable()) p.writer.join();
  p.writer_stop = false;
  std::lock_guard<std::mutex> g(p.m);
  for (auto* s : p.streams) {
    std::remove(s->spill_ev.c_str());
    std::remove(s->spill_info.c_str());
    delete s;
  }
  p.streams.clear();
  p.infos.clear();
  p.dict.clear();
  p.dict_index.clear();
  p.enabled = false;
  p.filename.clear();
  return 0;
}

void profiling_stream_add_information(ProfilingStream* s, const std::string& key, const std::string& value) {
  if (!s) return;
  std::lock_guard<SpinLock> g(s->lock);
  s->infos.emplace_back(key, value);
}

int profiling_dictionary_flush() {
  auto& p = P();
  std::lock_guard<std::mutex> g(p.m);
  p.dict.clear();
  p.dict_index.clear();
  return 0;
}

size_t profiling_key_info_length(int key) {
  auto& p = P();
  std::lock_guard<std::mutex> g(p.m);
  const size_t id = (size_t)(key / 2);
  return key >= 0 && id < p.dict.size() ? p.dict[id].info_length : 0;
}

void profiling_set_recording(bool on) { P().recording.store(on); }
const char* profiling_last_error() { return P().last_error.c_str(); }

void profiling_fini(Context* ctx) {
  auto& p = P();
  const auto ru = profiling_rusage();
  if (ParamRegistry::instance().reg_int("runtime", "", "report_rusage", "Print the process resource usage (getrusage) at fini", 0)) {
    std::string line;
    for (auto& kv : ru) line += " " + kv.first + "=" + std::to_string(kv.second);
    std::fprintf(stderr, "[parsec %d] rusage:%s\n", ctx->my_rank, line.c_str());
  }
  writer_drain();
  p.rank = ctx->my_rank;  // known only once the communication engine attached
  if (p.enabled && !p.filename.empty()) {
    for (auto& kv : ru) profiling_add_information(kv.first, std::to_string(kv.second));
    std::string fn = p.filename + "-" + std::to_string(ctx->my_rank) + ".prof";
    if (profiling_dump(fn) != 0) warning("could not write trace %s", fn.c_str());
  }
  {
    std::lock_guard<std::mutex> lk(p.wm);
    p.writer_stop = true;
  }
  p.wcv.notify_all();
  if (p.writer.joinable()) p.writer.join();
  p.writer_stop = false;
  std::lock_guard<std::mutex> g(p.m);
  for (auto* s : p.streams) {
    std::remove(s->spill_ev.c_str());
    std::remove(s->spill_info.c_str());
    delete s;
  }
  p.streams.clear();
  for (auto* es : ctx->all_es) es->prof = nullptr;
  for (auto* es : ctx->aux_es) es->prof = nullptr;
}

// ================================================================== PINS
std::atomic<bool> g_pins_enabled{false};
namespace {
struct PinsState {
  std::mutex m;
  std::vector<PinsCallback> cbs[PINS_NB_EVENTS];
  std::map<std::string, std::atomic<int64_t>*> counters;
  std::set<std::string> active;
};
PinsState& PS() { static PinsState* s = new PinsState(); return *s; }

std::atomic<int64_t>* counter(const std::string& n) {
  auto& s = PS();
  std::lock_guard<std::mutex> g(s.m);
  auto it = s.counters.find(n);
  if (it != s.counters.end()) return it->second;
  auto* c = new std::atomic<int64_t>(0);
  s.counters[n] = c;
  return c;
}

// task_profiler: one begin/end key per task class
constexpr int kProfiledLocals = 8;
int named_locals(const TaskClass* tc) {
  int n = std::min<int>({tc->nb_locals, (int)tc->local_names.size(), kProfiledLocals});
  for (int i = 0; i < n; ++i) {
    const std::string& nm = tc->local_names[i];
    bool ok = !nm.empty() && nm != "tp_id" && nm != "tc_id" && nm != "locals";
    for (char ch : nm) ok = ok && (std::isalnum((unsigned char)ch) || ch == '_');
    if (!ok) return i;
  }
  return n;
}
struct TaskProfiler {
  std::mutex m;
  std::map<const TaskClass*, std::pair<int, int>> keys;
  std::pair<int, int> key_of(const TaskClass* tc) {
    std::lock_guard<std::mutex> g(m);
    auto it = keys.find(tc);
    if (it != keys.end()) return it->second;
    int b, e;
    // the first two locals as an array, then every named local by its name
    // (what the reference's generated profiling convertors record: a column
    // per task parameter, e.g. "k" for ASYNC(k))
    std::string desc = "tp_id{uint32_t};tc_id{uint32_t};locals{int32_t[2]}";
    const int named = named_locals(tc);
    for (int i = 0; i < named; ++i) desc += ";" + tc->local_names[i] + "{int32_t}";
    profiling_add_dictionary_keyword(tc->name, "fill:#" + std::to_string(0x100000 + (tc->task_class_id * 2654435761u) % 0xEFFFFF), 16 + 4 * (size_t)named, desc, &b, &e);
    keys[tc] = {b, e};
    return {b, e};
  }
};
TaskProfiler& TPf() { static TaskProfiler* t = new TaskProfiler(); return *t; }
int g_key_release_b = -1, g_key_release_e = -1, g_key_select_b = -1, g_key_select_e = -1;
int g_key_activate_b = -1, g_key_activate_e = -1, g_key_flush_b = -1, g_key_flush_e = -1;
}  // namespace

void pins_fire(ExecutionStream* es, int event, Task* t) {
  auto& s = PS();
  for (auto& cb : s.cbs[event]) cb(es, event, t);
}

int pins_register_callback(int event, PinsCallback cb) {
  auto& s = PS();
  std::lock_guard<std::mutex> g(s.m);
  s.cbs[event].push_back(std::move(cb));
  g_pins_enabled.store(true);
  return 0;
}

std::vector<std::string> pins_modules_available() { return {"task_profiler", "print_steals", "alperf", "iterators_checker", "ptg_to_dtd"}; }

std::vector<std::pair<std::string, int64_t>> pins_counters() {
  auto& s = PS();
  std::lock_guard<std::mutex> g(s.m);
  std::vector<std::pair<std::string, int64_t>> out;
  for (auto& kv : s.counters) out.emplace_back(kv.first, kv.second->load());
  if (ptg_to_dtd_redirected() > 0) out.emplace_back("ptg_to_dtd.redirected", ptg_to_dtd_redirected());
  return out;
}

static void trace_task(ExecutionStream* es, Task* t, bool begin) {
  if (!es || !es->prof || !t) return;
  auto k = TPf().key_of(t->task_class);
  struct { uint32_t tp, tc; int32_t l[2]; int32_t named[kProfiledLocals]; } info{t->taskpool->taskpool_id, t->task_class->task_class_id,
                                                                               {t->locals[0], t->task_class->nb_locals > 1 ? t->locals[1] : 0}, {}};
  const int named = named_locals(t->task_class);
  for (int i = 0; i < named; ++i) info.named[i] = t->locals[i];
  profiling_trace(es->prof, begin ? k.first : k.second, t->key, t->taskpool->taskpool_id, &info, 16 + 4 * (size_t)named);
}

void pins_init(Context* ctx) {
  (void)ctx;
  std::string mods = ParamRegistry::instance().reg_string("mca", "", "pins", "Comma separated PINS modules: task_profiler,print_steals,alperf,iterators_checker,ptg_to_dtd", "");
  auto& s = PS();
  std::stringstream ss(mods);
  std::string m;
  while (std::getline(ss, m, ',')) {
    if (m.empty() || s.active.count(m)) continue;
    s.active.insert(m);
    if (m == "task_profiler") {
      profiling_add_dictionary_keyword("RELEASE_DEPS", "fill:#CCCCCC", 0, "", &g_key_release_b, &g_key_release_e);
      profiling_add_dictionary_keyword("SELECT", "fill:#EEEEEE", 0, "", &g_key_select_b, &g_key_select_e);
      pins_register_callback(PINS_EXEC_BEGIN, [](ExecutionStream* es, int, Task* t) { trace_task(es, t, true); });
      pins_register_callback(PINS_EXEC_END, [](ExecutionStream* es, int, Task* t) { trace_task(es, t, false); });
      pins_register_callback(PINS_COMPLETE_EXEC_BEGIN, [](ExecutionStream* es, int, Task* t) {
        if (es && es->prof) profiling_trace(es->prof, g_key_release_b, t ? t->key : 0, t ? t->taskpool->taskpool_id : 0, nullptr, 0);
      });
      pins_register_callback(PINS_COMPLETE_EXEC_END, [](ExecutionStream* es, int, Task*) {
        if (es && es->prof) profiling_trace(es->prof, g_key_release_e, 0, 0, nullptr, 0);
      });
      // remote activation callbacks (comm thread) and DTD data flushes
      profiling_add_dictionary_keyword("ACTIVATE_CB", "fill:#88CC88", 0, "", &g_key_activate_b, &g_key_activate_e);
      profiling_add_dictionary_keyword("DATA_FLUSH", "fill:#8888CC", 0, "", &g_key_flush_b, &g_key_flush_e);
      pins_register_callback(PINS_ACTIVATE_CB_BEGIN, [](ExecutionStream* es, int, Task*) {
        if (es && es->prof) profiling_trace(es->prof, g_key_activate_b, 0, 0, nullptr, 0);
      });
      pins_register_callback(PINS_ACTIVATE_CB_END, [](ExecutionStream* es, int, Task*) {
        if (es && es->prof) profiling_trace(es->prof, g_key_activate_e, 0, 0, nullptr, 0);
      });
      pins_register_callback(PINS_DATA_FLUSH_BEGIN, [](ExecutionStream* es, int, Task*) {
        if (es && es->prof) profiling_trace(es->prof, g_key_flush_b, 0, 0, nullptr, 0);
      });
      pins_register_callback(PINS_DATA_FLUSH_END, [](ExecutionStream* es, int, Task*) {
        if (es && es->prof) profiling_trace(es->prof, g_key_flush_e, 0, 0, nullptr, 0);
      });
    } else if (m == "print_steals") {
      pins_register_callback(PINS_THREAD_FINI, [](ExecutionStream* es, int, Task*) {
        counter("steals.thread" + std::to_string(es->th_id))->store((int64_t)es->nb_stolen);
        std::fprintf(stderr, "[print_steals] thread %d selected %llu stolen %llu\n", es->th_id, (unsigned long long)es->nb_selected, (unsigned long long)es->nb_stolen);
      });
    } else if (m == "alperf") {
      pins_register_callback(PINS_EXEC_END, [](ExecutionStream*, int, Task* t) {
        if (!t) return;
        counter("alperf.tp" + std::to_string(t->taskpool->taskpool_id) + "." + t->task_class->name)->fetch_add(1, std::memory_order_relaxed);
      });
    } else if (m == "iterators_checker") {
      pins_register_callback(PINS_EXEC_BEGIN, [](ExecutionStream* es, int, Task* t) {
        if (!t) return;
        // every local successor must list this task among its predecessors
        t->task_class->iterate_successors(es, t, ACTION_DEPS_MASK, [&](const DepVisit& v) {
          if (!v.tc) return;
          Task tmp;
          tmp.taskpool = t->taskpool;
          tmp.task_class = v.tc;
          for (int i = 0; i < v.nb_locals && i < kMaxLocals; ++i) tmp.locals[i] = v.locals[i];
          bool found = false;
          v.tc->iterate_predecessors(es, &tmp, ACTION_DEPS_MASK, [&](const DepVisit& p) {
            if (p.tc != t->task_class) return;
            bool same = true;
            for (int i = 0; i < t->task_class->nb_params; ++i) if (p.locals[i] != t->locals[i]) same = false;
            if (same) found = true;
          });
          counter(found ? "iterators_checker.ok" : "iterators_checker.mismatch")->fetch_add(1);
          if (!found) warning("iterators_checker: %s -> %s has no matching predecessor", t->task_class->describe(t).c_str(), v.tc->name.c_str());
        });
      });
    } else if (m == "ptg_to_dtd") {
      ptg_to_dtd_enable(true);
    } else {
      warning("unknown PINS module '%s'", m.c_str());
    }
  }
}

void pins_fini(Context* ctx) {
  (void)ctx;
  ptg_to_dtd_enable(false);
}

// ================================================================ grapher
namespace {
struct Grapher {
  std::mutex m;
  FILE* f = nullptr;
};
Grapher& G() { static Grapher* g = new Grapher(); return *g; }
std::string node_name(const TaskClass* tc, const int32_t* locals, int n) {
  std::string s = tc->name + "_";
  for (int i = 0; i < n; ++i) { if (i) s += "_"; s += std::to_string(locals[i]); }
  for (char& c : s) if (c == '-') c = 'm';
  return s;
}
}  // namespace

void grapher_init(Context* ctx) {
  if (ctx->grapher_file.empty()) return;
  auto& g = G();
  std::lock_guard<std::mutex> lk(g.m);
  std::string fn = ctx->grapher_file + "-" + std::to_string(ctx->my_rank) + ".dot";
  g.f = std::fopen(fn.c_str(), "w");
  if (g.f) std::fprintf(g.f, "digraph G {\n");
}

void grapher_task(ExecutionStream* es, Task* t) {
  (void)es;
  auto& g = G();
  if (!g.f) return;
  std::lock_guard<std::mutex> lk(g.m);
  std::fprintf(g.f, "  %s [label=\"%s\" tooltip=\"tp %u\"];\n", node_name(t->task_class, t->locals, t->task_class->nb_params).c_str(),
               t->task_class->describe(t).c_str(), t->taskpool->taskpool_id);
}

void grapher_dep(ExecutionStream* es, const Task* from, const TaskClass* to_tc, const int32_t* to_locals, int nb, int from_flow, int to_flow) {
  (void)es;
  auto& g = G();
  if (!g.f) return;
  std::lock_guard<std::mutex> lk(g.m);
  const char* fl = from_flow >= 0 && from_flow < (int)from->task_class->flows.size() ? from->task_class->flows[from_flow].name.c_str() : "";
  const char* tl = to_flow >= 0 && to_flow < (int)to_tc->flows.size() ? to_tc->flows[to_flow].name.c_str() : "";
  std::fprintf(g.f, "  %s -> %s [label=\"%s=>%s\"];\n", node_name(from->task_class, from->locals, from->task_class->nb_params).c_str(), node_name(to_tc, to_locals, nb).c_str(), fl, tl);
}

void grapher_fini(Context* ctx) {
  (void)ctx;
  auto& g = G();
  std::lock_guard<std::mutex> lk(g.m);
  if (g.f) { std::fprintf(g.f, "}\n"); std::fclose(g.f); g.f = nullptr; }
}

// ============================================================ properties
namespace {
struct Props { std::mutex m; std::map<std::string, double> v; };
Props& PR() { static Props* p = new Props(); return *p; }
}  // namespace

void properties_set(const std::string& name, double value) {
  auto& p = PR();
  std::lock_guard<std::mutex> g(p.m);
  p.v[name] = value;
}

std::vector<std::pair<std::string, double>> properties_snapshot() {
  auto& p = PR();
  std::lock_guard<std::mutex> g(p.m);
  std::vector<std::pair<std::string, double>> out(p.v.begin(), p.v.end());
  for (auto& c : pins_counters()) out.emplace_back(c.first, (double)c.second);
  return out;
}

// Runtime counters published next to the user properties: per-device
// executed tasks / kernel launches, threads and active taskpools,
// communication counters (reference dictionary.c namespaces
// PARSEC::<dev>::..., PARSEC::<thread>::...).
static std::vector<std::pair<std::string, double>> runtime_properties(Context* ctx) {
  std::vector<std::pair<std::string, double>> r;
  auto& reg = DeviceRegistry::instance();
  for (Device* d : reg.devices) {
    if (!d) continue;
    r.emplace_back("device." + d->name + ".executed_tasks", (double)d->stats.executed_tasks.load());
    r.emplace_back("device." + d->name + ".kernel_launches", (double)d->stats.kernel_launches.load());
  }
  if (ctx) {
    r.emplace_back("runtime.threads", (double)ctx->all_es.size());
    r.emplace_back("runtime.active_taskpools", (double)ctx->active_taskpools.load());
  }
  for (auto& kv : comm_stats()) r.emplace_back("comm." + kv.first, (double)kv.second);
  return r;
}

namespace {
struct Publisher {
  std::thread th;
  std::mutex m;
  std::condition_variable cv;
  bool stop = false;
  std::string name;
  Context* ctx = nullptr;
};
Publisher& PUB() { static Publisher* p = new Publisher(); return *p; }
}  // namespace

static int properties_write_shm(const std::string& shm_name, const std::vector<std::pair<std::string, double>>& snap, uint64_t seq);

// Live publication (reference aggregator_visu reads the dictionary from shm
// while the application runs): MCA profile_properties_shm=<name> refreshes
// /dev/shm/<name> every profile_properties_period_ms.
void properties_publisher_start(Context* ctx) {
  auto& pr = ParamRegistry::instance();
  std::string name = pr.reg_string("profile", "properties", "shm", "Publish runtime counters + properties in this POSIX shm segment while running", "");
  const int64_t period = pr.reg_int("profile", "properties", "period_ms", "Refresh period of the published properties (ms)", 100);
  if (name.empty()) return;
  if (name[0] != '/') name = "/" + name;
  auto& p = PUB();
  if (p.th.joinable()) return;
  p.stop = false;
  p.name = name;
  p.ctx = ctx;
  p.th = std::thread([&p, period] {
    uint64_t seq = 0;
    std::unique_lock<std::mutex> lk(p.m);
    for (;;) {
      auto snap = properties_snapshot();
      for (auto& kv : runtime_properties(p.ctx)) snap.push_back(kv);
      properties_write_shm(p.name, snap, ++seq);
      if (p.cv.wait_for(lk, std::chrono::milliseconds(std::max<int64_t>(period, 1)), [&] { return p.stop; })) break;
    }
  });
}

void properties_publisher_stop() {
  auto& p = PUB();
  if (!p.th.joinable()) return;
  {
    std::lock_guard<std::mutex> g(p.m);
    p.stop = true;
  }
  p.cv.notify_all();
  p.th.join();
  // final values stay readable after the run; the segment is the user's to remove
  auto snap = properties_snapshot();
  for (auto& kv : runtime_properties(p.ctx)) snap.push_back(kv);
  properties_write_shm(p.name, snap, ~0ull);
  p.ctx = nullptr;
}

int properties_dump_shm(const std::string& shm_name) { return properties_write_shm(shm_name, properties_snapshot(), 0); }

// Publish properties in a POSIX shm region: an XML-ish header then the values
// (reference dictionary.c exposes the same through shm for aggregator_visu).
static int properties_write_shm(const std::string& shm_name, const std::vector<std::pair<std::string, double>>& snap, uint64_t seq) {
  std::ostringstream os;
  os << "<properties seq=\"" << seq << "\">\n";
  for (auto& kv : snap) os << "  <p name=\"" << kv.first << "\" value=\"" << kv.second << "\"/>\n";
  os << "</properties>\n";
  std::string s = os.str();
  int fd = shm_open(shm_name.c_str(), O_CREAT | O_RDWR, 0600);
  if (fd < 0) return -1;
  if (ftruncate(fd, (off_t)s.size() + 1) != 0) { close(fd); return -1; }
  void* p = mmap(nullptr, s.size() + 1, PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return -1;
  std::memcpy(p, s.c_str(), s.size() + 1);
  munmap(p, s.size() + 1);
  return 0;
}

}  // namespace parsec
