#include <array>
// Context bring-up / tear-down, virtual-process map, thread binding.
//
// Parity: parsec_init/parsec_fini (reference parsec.c:384-924, 1158-1301),
// vpmap flat | rr:n:p:c | file: (vpmap.c:162-443), thread binding (bindthread.c:35-110),
// context start/wait/test epochs (scheduling.c:537-808).
// Design: the calling thread is compute thread 0; the others are std::threads
// that sleep on a condition variable between epochs. Steal order is derived from
// the Linux /sys topology (package + NUMA node) instead of hwloc.
#include <execinfo.h>
#include <csignal>
#include <unistd.h>
#include <pthread.h>
#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <fstream>
#include <sstream>

#include "../comm/comm.hpp"
#include "../device/device.hpp"
#include "../prof/profiling.hpp"
#include "runtime.hpp"

namespace parsec {

static thread_local ExecutionStream* t_es = nullptr;
static std::atomic<int> g_next_slot{0};

int thread_slot() {
  thread_local int slot = -1;
  if (slot < 0) {
    slot = g_next_slot.fetch_add(1);
    if (slot >= kMaxThreadSlots) fatal("too many threads touching the runtime (%d)", slot);
  }
  return slot;
}
ExecutionStream* my_execution_stream() { return t_es; }
void set_my_execution_stream(ExecutionStream* es) { t_es = es; }

// ----------------------------------------------------------- topology
// hwloc-equivalent view of one allowed CPU (reference parsec_hwloc.c): the
// package, NUMA node and the caches it shares (id = lowest CPU sharing it)
struct CpuTopo {
  int cpu;
  int package;
  int numa;
  int l2 = -1, l3 = -1;
};

static int first_cpu_of_list(const std::string& path) {
  std::ifstream in(path);
  std::string s;
  if (!(in >> s)) return -1;
  return std::atoi(s.c_str());  // "a-b,c..." -> a
}

static int read_int_file(const std::string& p, int dflt) {
  std::ifstream in(p);
  int v;
  if (in >> v) return v;
  return dflt;
}

static std::vector<CpuTopo> allowed_cpus() {
  std::vector<CpuTopo> out;
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) != 0) {
    int n = (int)std::thread::hardware_concurrency();
    for (int i = 0; i < n; ++i) out.push_back({i, 0, 0});
    return out;
  }
  for (int c = 0; c < CPU_SETSIZE; ++c) {
    if (!CPU_ISSET(c, &set)) continue;
    CpuTopo t{c, 0, 0};
    t.package = read_int_file("/sys/devices/system/cpu/cpu" + std::to_string(c) + "/topology/physical_package_id", 0);
    // NUMA node: look for nodeN link
    for (int n = 0; n < 16; ++n) {
      std::ifstream probe("/sys/devices/system/cpu/cpu" + std::to_string(c) + "/node" + std::to_string(n) + "/cpumap");
      if (probe) { t.numa = n; break; }
    }
    for (int k = 0; k < 8; ++k) {
      const std::string base = "/sys/devices/system/cpu/cpu" + std::to_string(c) + "/cache/index" + std::to_string(k) + "/";
      const int level = read_int_file(base + "level", -1);
      if (level < 0) break;
      if (level == 2) t.l2 = first_cpu_of_list(base + "shared_cpu_list");
      if (level == 3) t.l3 = first_cpu_of_list(base + "shared_cpu_list");
    }
    out.push_back(t);
  }
  return out;
}

std::vector<std::array<int, 5>> topology_cpus() {
  std::vector<std::array<int, 5>> r;
  for (auto& c : allowed_cpus()) r.push_back({c.cpu, c.package, c.numa, c.l2, c.l3});
  return r;
}

std::vector<std::vector<int>> topology_numa_distances() {
  std::vector<std::vector<int>> r;
  for (int n = 0; n < 64; ++n) {
    std::ifstream in("/sys/devices/system/node/node" + std::to_string(n) + "/distance");
    if (!in) break;
    std::vector<int> row;
    int v;
    while (in >> v) row.push_back(v);
    r.push_back(row);
  }
  return r;
}

static void bind_current_thread(int cpu) {
  if (cpu < 0) return;
  cpu_set_t set;
  CPU_ZERO(&set);
  CPU_SET(cpu, &set);
  if (pthread_setaffinity_np(pthread_self(), sizeof(set), &set) != 0)
    PARSEC_DEBUG(kVerbInfo, "bind", "could not bind thread to core %d", cpu);
}

// Parse the vpmap: "flat" (default), "rr:n:p:c" (n VPs of p threads...), "file:<path>"
// (one line per VP listing its core ids), "vps:<n>" (n equal VPs).
static std::vector<std::vector<int>> build_vpmap(const std::string& spec, int nb_cores) {
  std::vector<std::vector<int>> vps;
  if (spec.rfind("file:", 0) == 0) {
    std::ifstream in(spec.substr(5));
    std::string line;
    int tid = 0;
    while (std::getline(in, line) && tid < nb_cores) {
      std::stringstream ss(line);
      std::vector<int> vp;
      int c;
      while (ss >> c && tid < nb_cores) { vp.push_back(tid++); (void)c; }
      if (!vp.empty()) vps.push_back(vp);
    }
    for (; tid < nb_cores; ++tid) { if (vps.empty()) vps.emplace_back(); vps.back().push_back(tid); }
  } else if (spec.rfind("rr:", 0) == 0 || spec.rfind("vps:", 0) == 0) {
    int n = std::max(1, std::atoi(spec.substr(spec.find(':') + 1).c_str()));
    n = std::min(n, nb_cores);
    vps.resize(n);
    for (int t = 0; t < nb_cores; ++t) vps[t * n / nb_cores].push_back(t);
  } else {
    vps.emplace_back();
    for (int t = 0; t < nb_cores; ++t) vps[0].push_back(t);
  }
  return vps;
}

// ----------------------------------------------------------- threads
static void thread_main(Context* ctx, ExecutionStream* es) {
  set_my_execution_stream(es);
  es->slot = thread_slot();
  if (!ctx->core_bindings.empty()) bind_current_thread(ctx->core_bindings[es->th_id % ctx->core_bindings.size()]);
  ctx->scheduler->flow_init(es, ctx->barrier);
  profiling_thread_init(es);
  PARSEC_PINS(es, PINS_THREAD_INIT, nullptr);
  ctx->barrier->wait();
  uint64_t seen_epoch = 0;
  for (;;) {
    {
      std::unique_lock<std::mutex> g(ctx->wake_m);
      ctx->wake_cv.wait(g, [&] { return ctx->finalizing.load() || (ctx->started.load() && ctx->epoch.load() != seen_epoch); });
      if (ctx->finalizing.load()) break;
      seen_epoch = ctx->epoch.load();
    }
    worker_loop(es, false);
  }
  PARSEC_PINS(es, PINS_THREAD_FINI, nullptr);
  profiling_thread_fini(es);
}

// Fatal-signal handler (reference debug_backtrace_* MCA params, utils/debug.c):
// print the faulting rank and a native backtrace, then re-raise.
static void fatal_signal_handler(int sig) {
  char head[96];
  int n = std::snprintf(head, sizeof(head), "[parsec %d] fatal signal %d, backtrace:\n", debug_rank(), sig);
  if (n > 0) (void)!write(2, head, (size_t)n);
  void* frames[64];
  int k = backtrace(frames, 64);
  backtrace_symbols_fd(frames, k, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

static void install_fatal_handlers() {
  static std::atomic<bool> done{false};
  if (done.exchange(true)) return;
  if (!ParamRegistry::instance().reg_int("debug", "", "backtrace_on_fatal", "Print a native backtrace on SIGSEGV / SIGBUS / SIGABRT / SIGFPE", 1)) return;
  for (int s : {SIGSEGV, SIGBUS, SIGFPE, SIGABRT}) signal(s, fatal_signal_handler);
}

Context* context_init(int nb_cores, std::vector<std::string>& args) {
  install_fatal_handlers();
  auto& reg = ParamRegistry::instance();
  args = reg.parse_cmdline(args);
  output_init();
  Context* ctx = new Context();
  context_set_live(ctx, true);

  int param_cores = (int)reg.reg_int("runtime", "", "num_cores", "Number of compute threads (0 = all allowed cores)", 0);
  auto cpus = allowed_cpus();
  if (nb_cores <= 0) nb_cores = param_cores > 0 ? param_cores : (int)cpus.size();
  if (nb_cores <= 0) nb_cores = 1;
  ctx->nb_cores = nb_cores;
  ctx->keep_highest_priority_task = reg.reg_int("runtime", "", "keep_highest_priority_task", "Keep the highest priority ready task on the releasing thread", 1) != 0;
  ctx->paranoid = reg.reg_int("debug", "", "paranoid", "Check task lifecycle invariants (scheduled twice, completed twice, scheduled after release, PTG dependency underflow)", 0) != 0;
  g_paranoid = ctx->paranoid;
  {
    int im = (int)reg.reg_int("device", "", "manager_inline_dispatch", "GPU managers (and the comm thread) prepare and submit successors whose first chore is a GPU chore: 0 off, 1 managers + comm, 2 managers only, 3 comm only", 1);
    ctx->manager_inline_gpu = im != 0;
    ctx->manager_inline_mode = im;
  }
  std::string bcast = reg.reg_string("runtime", "comm", "coll_bcast", "Broadcast topology for remote activations: star|chain|binomial", "star");
  ctx->comm_bcast_topology = bcast == "chain" ? 1 : bcast == "binomial" ? 2 : 0;
  ctx->default_termdet = reg.reg_string("termdet", "", "default", "Default termination detection module", "local");
  ctx->grapher_file = reg.reg_string("parsec", "", "dot", "Write the executed DAG as a DOT file (prefix)", "");
  ctx->simulation = reg.reg_int("runtime", "", "simulation", "Compute the critical path length (simulation mode)", 0) != 0;

  bool bind = reg.reg_int("runtime", "", "bind_threads", "Bind compute threads to cores", 0) != 0;
  if (bind) for (auto& c : cpus) ctx->core_bindings.push_back(c.cpu);

  // virtual processes
  std::string vpmap = reg.reg_string("runtime", "", "vpmap", "Virtual-process map: flat | vps:<n> | rr:<n>[:p:c] | file:<path>", "flat");
  auto vps = build_vpmap(vpmap, nb_cores);
  ctx->nb_vp = (int)vps.size();
  for (int v = 0; v < ctx->nb_vp; ++v) {
    auto* vp = new VirtualProcess();
    vp->parsec_context = ctx;
    vp->vp_id = v;
    for (int tid : vps[v]) {
      auto* es = new ExecutionStream();
      es->th_id = tid;
      es->virtual_process = vp;
      es->ctx = ctx;
      es->rand_seed = 1234567u + 7919u * tid;
      if (!cpus.empty()) {
        const CpuTopo& ct = cpus[tid % cpus.size()];
        es->core_id = ct.cpu;
        es->socket_id = ct.package * 64 + ct.numa;
        es->l2_id = ct.l2;
        es->l3_id = ct.l3;
      }
      vp->es.push_back(es);
      vp->nb_cores = (int)vp->es.size();
      ctx->all_es.push_back(es);
    }
    ctx->vps.push_back(vp);
  }
  std::sort(ctx->all_es.begin(), ctx->all_es.end(), [](auto* a, auto* b) { return a->th_id < b->th_id; });
  // steal order: same VP only (no stealing across VPs), closest first in the
  // cache hierarchy: shared L2, shared L3, same NUMA node, same package, other
  for (auto* vp : ctx->vps)
    for (auto* es : vp->es) {
      std::vector<std::pair<int, int>> d;
      for (auto* o : vp->es) {
        if (o == es) continue;
        int dist = 4;
        if (o->l2_id >= 0 && o->l2_id == es->l2_id) dist = 0;
        else if (o->l3_id >= 0 && o->l3_id == es->l3_id) dist = 1;
        else if (o->socket_id == es->socket_id) dist = 2;
        else if (o->socket_id / 64 == es->socket_id / 64) dist = 3;
        d.push_back({dist, o->th_id});
      }
      std::stable_sort(d.begin(), d.end());
      // rotate within each equal-distance group so threads do not all hit the
      // same victim first (the groups themselves stay in distance order)
      for (size_t b = 0; b < d.size();) {
        size_t e = b;
        while (e < d.size() && d[e].first == d[b].first) ++e;
        const size_t n = e - b;
        if (n > 1) std::rotate(d.begin() + b, d.begin() + b + (size_t)es->th_id % n, d.begin() + e);
        b = e;
      }
      for (auto& p : d) es->steal_order.push_back(p.second);
    }

  // task mempool: large enough for every front-end's task type.
  ctx->task_size = std::max<size_t>(sizeof(Task), 1024);
  ctx->task_mempool = std::make_unique<Mempool>(ctx->task_size, kMaxThreadSlots);

  // scheduler
  std::string want = reg.reg_string("mca", "", "sched", "Scheduler to use (lfq, pbq, ltq, lhq, ap, spq, gd, ll, llp, rnd, ip)", "");
  const SchedulerComponent* best = nullptr;
  for (auto& c : scheduler_components()) {
    if (!want.empty()) { if (want == c.name) best = &c; }
    else if (!best || c.priority > best->priority) best = &c;
  }
  if (!best) fatal("scheduler '%s' not found", want.c_str());
  ctx->scheduler = best->factory();
  ctx->scheduler_name = best->name;
  ctx->scheduler->install(ctx);

  // ranks (comm engine attaches later via remote_dep_init)
  profiling_init(ctx);
  pins_init(ctx);
  devices_init(ctx);
  remote_dep_init(ctx);
  properties_publisher_start(ctx);

  // threads
  ctx->barrier = new Barrier(nb_cores);
  ExecutionStream* master = ctx->all_es[0];
  for (int t = 1; t < nb_cores; ++t) ctx->threads.emplace_back(thread_main, ctx, ctx->all_es[t]);
  set_my_execution_stream(master);
  master->slot = thread_slot();
  if (!ctx->core_bindings.empty() && reg.reg_int("runtime", "", "bind_main_thread", "Bind the main thread", 0)) bind_current_thread(ctx->core_bindings[0]);
  ctx->scheduler->flow_init(master, ctx->barrier);
  profiling_thread_init(master);
  PARSEC_PINS(master, PINS_THREAD_INIT, nullptr);
  ctx->barrier->wait();
  devices_start(ctx);
  grapher_init(ctx);
  PARSEC_DEBUG(kVerbInfo, "init", "context up: %d threads, %d vp, scheduler %s, %d devices, rank %d/%d", nb_cores, ctx->nb_vp,
               ctx->scheduler_name.c_str(), DeviceRegistry::instance().count(), ctx->my_rank, ctx->nb_nodes);
  return ctx;
}

int context_fini(Context** pctx) {
  Context* ctx = *pctx;
  if (!ctx) return 0;
  if (ctx->active_taskpools.load() > 0) context_wait(ctx);
  context_drain_zombies(ctx);
  PARSEC_DEBUG(kVerbDebug, "fini", "at_fini hooks (%zu)", ctx->at_fini.size());
  for (size_t i = 0; i < ctx->at_fini.size(); ++i) ctx->at_fini[i](ctx->at_fini_data[i]);
  PARSEC_DEBUG(kVerbDebug, "fini", "remote deps");
  remote_dep_fini(ctx);
  PARSEC_DEBUG(kVerbDebug, "fini", "devices stop");
  devices_stop(ctx);
  PARSEC_DEBUG(kVerbDebug, "fini", "joining workers");
  {
    std::lock_guard<std::mutex> g(ctx->wake_m);
    ctx->finalizing.store(true);
  }
  ctx->wake_cv.notify_all();
  for (auto& t : ctx->threads) t.join();
  ctx->threads.clear();
  PARSEC_DEBUG(kVerbDebug, "fini", "workers joined");
  ExecutionStream* master = ctx->all_es[0];
  PARSEC_PINS(master, PINS_THREAD_FINI, nullptr);
  if (ParamRegistry::instance().reg_int("runtime", "", "show_stats", "Display scheduler statistics at fini", 0))
    for (auto* es : ctx->all_es) ctx->scheduler->display_stats(es);
  profiling_thread_fini(master);
  grapher_fini(ctx);
  pins_fini(ctx);
  properties_publisher_stop();
  profiling_fini(ctx);
  PARSEC_DEBUG(kVerbDebug, "fini", "devices fini");
  devices_fini(ctx);
  PARSEC_DEBUG(kVerbDebug, "fini", "scheduler remove");
  ctx->scheduler->remove(ctx);
  delete ctx->scheduler;
  // manager / comm pseudo execution streams (their threads are stopped by now)
  for (auto* es : ctx->aux_es) delete es;
  ctx->aux_es.clear();
  for (auto* vp : ctx->vps) {
    for (auto* es : vp->es) delete es;
    delete vp;
  }
  delete ctx->barrier;
  set_my_execution_stream(nullptr);
  context_set_live(ctx, false);
  delete ctx;
  *pctx = nullptr;
  PARSEC_DEBUG(kVerbDebug, "fini", "context released");
  return 0;
}

void context_abort(Context* ctx, int status) {
  (void)ctx;
  std::fprintf(stderr, "[parsec] abort(%d)\n", status);
  std::fflush(stderr);
  std::_Exit(status ? status : 1);
}

int context_start(Context* ctx) {
  remote_dep_on(ctx);
  {
    std::lock_guard<std::mutex> g(ctx->wake_m);
    ctx->started.store(true);
    ctx->epoch.fetch_add(1);
  }
  ctx->wake_cv.notify_all();
  return 0;
}

int context_test(Context* ctx) { return ctx->active_taskpools.load() == 0 ? 1 : 0; }

int context_wait(Context* ctx) {
  if (!ctx->started.load()) context_start(ctx);
  ExecutionStream* es = my_execution_stream();
  if (!es || es->ctx != ctx) es = ctx->all_es[0];
  ExecutionStream* prev = my_execution_stream();
  set_my_execution_stream(es);
  std::vector<Taskpool*> tps;
  {
    std::lock_guard<std::mutex> g(ctx->tp_m);
    tps = ctx->taskpools_in_flight;
  }
  for (Taskpool* tp : tps) tp->on_context_wait();
  worker_loop(es, true);
  context_drain_zombies(ctx);
  set_my_execution_stream(prev);
  {
    std::lock_guard<std::mutex> g(ctx->wake_m);
    ctx->started.store(false);
  }
  remote_dep_off(ctx);
  return 0;
}

}  // namespace parsec
