// Device registry, CPU and recursive devices, load-balanced device selection,
// CPU-side staging of device-resident data.
//
// Parity: reference mca/device/device.c (registry :194-285, attach :843-904,
// registration_complete -> relative weights :617-666, CPU weights :678-797,
// parsec_get_best_device :79-189 with load_balance_skew).
#include "device.hpp"

#include <fstream>

#include <unistd.h>

#include <cmath>
#include <cstdlib>
#include <cstring>

#include "hip_device.hpp"

namespace parsec {

DeviceRegistry& DeviceRegistry::instance() {
  static DeviceRegistry* r = new DeviceRegistry();
  return *r;
}

int DeviceRegistry::add(Device* d) {
  d->device_index = (int)devices.size();
  devices.push_back(d);
  return d->device_index;
}

int DeviceRegistry::nb_gpus() const {
  int n = 0;
  for (auto* d : devices) if (d && d->is_gpu()) ++n;
  return n;
}

void DeviceRegistry::registration_complete() {
  double maxg = 0;
  for (auto* d : devices) if (d) maxg = std::max(maxg, d->gflops_fp64);
  for (auto* d : devices) if (d) d->gflops_weight = d->gflops_fp64 > 0 ? maxg / d->gflops_fp64 : 1e9;
  frozen = true;
}

// CPU capability (reference device.c:678-797 parses /proc/cpuinfo for the
// clock and the widest vector ISA): peak fp64 flops per cycle and core from the
// ISA flags, the clock from cpufreq (max) or the "cpu MHz" lines.
CpuCapability cpu_capability() {
  CpuCapability c;
  std::ifstream f("/proc/cpuinfo");
  std::string line;
  double mhz = 0;
  while (std::getline(f, line)) {
    const auto colon = line.find(':');
    if (colon == std::string::npos) continue;
    std::string key = line.substr(0, colon);
    while (!key.empty() && (key.back() == ' ' || key.back() == '\t')) key.pop_back();
    const std::string val = line.substr(colon + 1);
    if (key == "model name" && c.model.empty()) c.model = val.substr(val.find_first_not_of(' ') == std::string::npos ? 0 : val.find_first_not_of(' '));
    else if (key == "cpu MHz") mhz = std::max(mhz, std::atof(val.c_str()));
    else if (key == "flags" && c.flags_seen == false) {
      c.flags_seen = true;
      auto has = [&](const char* fl) { return (" " + val + " ").find(std::string(" ") + fl + " ") != std::string::npos; };
      c.avx512 = has("avx512f");
      c.avx2 = has("avx2");
      c.fma = has("fma");
      c.sse2 = has("sse2");
    }
  }
  std::ifstream fq("/sys/devices/system/cpu/cpu0/cpufreq/cpuinfo_max_freq");
  long khz = 0;
  if (fq >> khz && khz > 0) mhz = std::max(mhz, khz / 1000.0);
  c.ghz = mhz > 0 ? mhz / 1000.0 : 2.0;
  // 2 FMA pipes x vector doubles x 2 flops
  c.dp_flops_per_cycle = c.avx512 ? 32.0 : (c.avx2 && c.fma) ? 16.0 : c.avx2 ? 8.0 : c.sse2 ? 4.0 : 2.0;
  if (c.isa().empty()) c.model = c.model.empty() ? "unknown" : c.model;
  return c;
}

std::string CpuCapability::isa() const { return avx512 ? "AVX512" : (avx2 && fma) ? "AVX2+FMA" : avx2 ? "AVX2" : sse2 ? "SSE2" : "scalar"; }

struct CpuDevice : Device {
  CpuCapability cap;
  CpuDevice(int cores) : cap(cpu_capability()) {
    name = "cpu";
    type = DEV_CPU;
    gflops_fp64 = std::max(1, cores) * cap.ghz * cap.dp_flops_per_cycle;
    gflops_fp32 = 2 * gflops_fp64;
    PARSEC_DEBUG(kVerbInfo, "device", "cpu: %s, %s at %.2f GHz: %.1f GFLOP/s fp64 over %d cores", cap.model.c_str(), cap.isa().c_str(), cap.ghz, gflops_fp64, cores);
  }
};

struct RecursiveDevice : Device {
  RecursiveDevice() { name = "recursive"; type = DEV_RECURSIVE; gflops_fp64 = 1; }
};

// Device template (reference mca/device/template): a pseudo-accelerator whose
// chores (type DEV_TEMPLATE) run on the worker threads, with no-op memory
// registration. It exercises chore selection, device masks and per-device
// statistics without GPU hardware (--mca device_template_enabled 1).
struct TemplateDevice : Device {
  TemplateDevice() { name = "template"; type = DEV_TEMPLATE; gflops_fp64 = 1; }
  int memory_register(DataCollection*, void*, size_t) override { return 0; }
  int memory_unregister(DataCollection*, void*) override { return 0; }
};

static double g_load_balance_skew = 20.0;

void devices_init(Context* ctx) {
  auto& reg = DeviceRegistry::instance();
  auto& params = ParamRegistry::instance();
  g_load_balance_skew = (double)params.reg_int("device", "", "load_balance_skew", "Allowed load imbalance (percent) before moving work off the data-owner device", 20);
  const double cpu_g = (double)params.reg_int("device", "cpu", "gflops", "Override the CPU device fp64 GFLOP/s estimate (0 = estimate)", 0);
  if (reg.devices.empty()) {
    auto* cpu = new CpuDevice(ctx->nb_cores);
    if (cpu_g > 0) cpu->gflops_fp64 = cpu_g;
    reg.add(cpu);
    reg.add(new RecursiveDevice());
    hip_devices_init(ctx);
    reg.registration_complete();
  } else {
    // the registry outlives a context: a later context's core count sets the
    // CPU device's capability (and so the weights) again
    for (auto* d : reg.devices)
      if (d && d->type == DEV_CPU) {
        auto* cpu = static_cast<CpuDevice*>(d);
        cpu->gflops_fp64 = cpu_g > 0 ? cpu_g : std::max(1, ctx->nb_cores) * cpu->cap.ghz * cpu->cap.dp_flops_per_cycle;
        cpu->gflops_fp32 = 2 * cpu->gflops_fp64;
      }
    reg.registration_complete();
  }
  // the template device can be enabled by a later context of the same process
  if (params.reg_int("device", "template", "enabled", "Register the template pseudo-device (framework testing)", 0)) {
    bool have = false;
    for (auto* d : reg.devices) if (d && d->type == DEV_TEMPLATE) have = true;
    if (!have) {
      reg.add(new TemplateDevice());
      reg.registration_complete();
    }
  }
  for (auto* d : reg.devices) if (d) d->attach(ctx);
  if (params.reg_int("device", "", "show_capabilities", "Print device capabilities at init", 0))
    for (auto* d : reg.devices)
      if (d) std::fprintf(stderr, "[parsec] device %d %s type=0x%x fp64=%.0f GF weight=%.3f\n", d->device_index, d->name.c_str(), d->type, d->gflops_fp64, d->gflops_weight);
}

void devices_start(Context* ctx) { hip_devices_start(ctx); }
void devices_stop(Context* ctx) { hip_devices_stop(ctx); }

void devices_fini(Context* ctx) {
  auto& reg = DeviceRegistry::instance();
  if (ParamRegistry::instance().reg_int("device", "", "show_statistics", "Print per-device statistics at fini", 0)) {
    for (auto* d : reg.devices) {
      if (!d) continue;
      std::fprintf(stderr, "[parsec] device %d %-10s tasks=%llu launches=%llu batched=%llu in=%llu B out=%llu B d2d=%llu B faults=%llu\n", d->device_index, d->name.c_str(),
                   (unsigned long long)d->stats.executed_tasks.load(), (unsigned long long)d->stats.kernel_launches.load(), (unsigned long long)d->stats.batched_tasks.load(),
                   (unsigned long long)d->stats.bytes_in.load(), (unsigned long long)d->stats.bytes_out.load(), (unsigned long long)d->stats.bytes_d2d.load(),
                   (unsigned long long)d->stats.data_faults.load());
    }
  }
  for (auto* d : reg.devices) if (d) d->detach(ctx);
}

bool device_type_enabled(Taskpool* tp, uint32_t type) {
  auto& reg = DeviceRegistry::instance();
  for (auto* d : reg.devices) {
    if (!d || !(d->type & type)) continue;
    if (tp->devices_index_mask & (1u << d->device_index)) return true;
  }
  return false;
}

int get_best_device(Task* t, double ratio) {
  auto& reg = DeviceRegistry::instance();
  Taskpool* tp = t->taskpool;
  const TaskClass* tc = t->task_class;
  int dev = -1;
  // 1) locality: a device that owns (or prefers) data we write, then data we read
  for (int pass = 0; pass < 2 && dev < 0; ++pass) {
    for (auto& f : tc->flows) {
      if (f.access == FLOW_CTL || f.access == FLOW_NONE) continue;
      bool w = f.access & FLOW_WRITE;
      if ((pass == 0) != w) continue;
      DataCopy* c = t->data[f.index].data_in;
      if (!c || !c->original) continue;
      Data* d = c->original;
      int cand = d->preferred_device >= 2 ? d->preferred_device : d->owner_device;
      if (cand >= 2 && cand < reg.count() && reg.devices[cand] && reg.devices[cand]->is_gpu() && (tp->devices_index_mask & (1u << cand))) {
        dev = cand;
        break;
      }
    }
  }
  // 2) load balance among enabled GPUs; keep the locality choice unless skewed
  int best = -1;
  double best_load = 0;
  for (auto* d : reg.devices) {
    if (!d || !d->is_gpu() || !(tp->devices_index_mask & (1u << d->device_index))) continue;
    double l = (double)d->load.load(std::memory_order_relaxed) + ratio * d->gflops_weight;
    if (best < 0 || l < best_load) { best = d->device_index; best_load = l; }
  }
  if (dev >= 0 && best >= 0 && dev != best) {
    double ldev = (double)reg.devices[dev]->load.load() + ratio * reg.devices[dev]->gflops_weight;
    if (ldev <= best_load * (1.0 + g_load_balance_skew / 100.0) + 1) return dev;
    return best;
  }
  return dev >= 0 ? dev : best;
}

int gpu_chore_dispatch(ExecutionStream* es, Task* t, int chore) {
  const Chore& ch = t->task_class->chores[chore];
  int dev = t->selected_device >= 2 ? t->selected_device : get_best_device(t, ch.weight_of(t));
  if (dev < 2) return HOOK_NEXT;
  t->selected_device = (int8_t)dev;
  return DeviceRegistry::instance().devices[dev]->submit(es, t, chore);
}

// ------------------------------------------------------------ host staging
DataCopy* data_pull_to_host(Data* d) {
  if (!d) return nullptr;
  DataCopy* host = d->copy(0);
  if (!host) {
    void* p = nullptr;
    if (posix_memalign(&p, 4096, std::max<size_t>(d->nb_elts, 64))) fatal("host allocation failed");
    DataCopy* c = new DataCopy();
    c->device_private = p;
    c->flags = DATA_FLAG_PARSEC_OWNED;
    c->coherency_state = COHERENCY_INVALID;
    c->version = 0;
    std::lock_guard<SpinLock> g(d->lock);
    if (!d->copy(0)) data_copy_attach(d, c, 0);
    else { std::free(p); delete c; }
    host = d->copy(0);
  }
  DataCopy* src = data_start_transfer_ownership_to_copy(d, 0, FLOW_READ);
  bool pinned = false;
  if (src && src != host && src->device_index != 0) src = pin_gpu_source(d, 0, host, src, FLOW_READ, &pinned);
  if (src && src != host) {
    device_memcpy(0, host->device_private, src->device_index, src->device_private, d->nb_elts);
    auto* dev = DeviceRegistry::instance().get(src->device_index);
    if (dev) dev->stats.bytes_out.fetch_add(d->nb_elts, std::memory_order_relaxed);
  }
  if (pinned) unpin_gpu_copy(src);
  data_end_transfer_ownership_to_copy(d, 0, FLOW_READ);
  return host;
}

void cpu_stage_in(ExecutionStream* es, Task* t) {
  (void)es;
  for (auto& f : t->task_class->flows) {
    if (f.access == FLOW_CTL || f.access == FLOW_NONE) continue;
    TaskDataRef& r = t->data[f.index];
    DataCopy* c = r.data_in;
    // an early-released GPU group may still be writing (or reading) this copy
    if (c)
      if (void* ev = c->pending_event.load(std::memory_order_acquire)) (void)hipEventSynchronize((hipEvent_t)ev);
    if (!c || !c->original) continue;
    Data* d = c->original;
    bool needs = c->device_index != 0;
    if (!needs) {
      // host copy present: is it current?
      std::lock_guard<SpinLock> g(d->lock);
      uint32_t newest = 0;
      for (int i = 1; i < kMaxDevices; ++i) { DataCopy* o = d->copy(i); if (o && o->coherency_state != COHERENCY_INVALID) newest = std::max<uint32_t>(newest, o->version); }
      needs = newest > c->version && (f.access & FLOW_READ);
    }
    if (!needs) continue;
    DataCopy* host = data_pull_to_host(d);
    if (host != c) {
      data_copy_retain(host);
      data_copy_release(c);
      r.data_in = host;
    }
  }
}

void cpu_write_epilog(Task* t) {
  for (auto& f : t->task_class->flows) {
    if (!(f.access & FLOW_WRITE)) continue;
    DataCopy* c = t->data[f.index].data_in;
    if (!c || !c->original || c->device_index != 0) continue;
    Data* d = c->original;
    std::lock_guard<SpinLock> g(d->lock);
    uint32_t v = 0;
    for (int i = 0; i < kMaxDevices; ++i) { DataCopy* o = d->copy(i); if (o && o->coherency_state != COHERENCY_INVALID) v = std::max<uint32_t>(v, o->version); }
    c->version = v + 1;
    c->coherency_state = COHERENCY_OWNED;
    d->owner_device = 0;
  }
}

int device_hip_ordinal(int device_index) {
  auto* d = DeviceRegistry::instance().get(device_index);
  if (!d || !d->is_gpu()) return -1;
  return static_cast<HipDevice*>(d)->ordinal;
}

int first_gpu_device_index() {
  for (auto* d : DeviceRegistry::instance().devices) if (d && d->is_gpu()) return d->device_index;
  return -1;
}

int data_advise_on_device(Data* d, int device_index, int advice) {
  auto& reg = DeviceRegistry::instance();
  if (!d || device_index < 0 || device_index >= reg.count() || !reg.devices[device_index]) return -1;
  if (advice == DATA_ADVICE_PREFERRED_DEVICE) d->preferred_device = (int8_t)device_index;
  reg.devices[device_index]->data_advise(d, advice);
  return 0;
}

}  // namespace parsec
