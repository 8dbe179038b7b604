#include "mca.hpp"

#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

namespace parsec {

ParamRegistry& ParamRegistry::instance() {
  static ParamRegistry* r = new ParamRegistry();
  return *r;
}

std::string ParamRegistry::join(const std::string& type, const std::string& comp, const std::string& name) {
  std::string s;
  for (const std::string* p : {&type, &comp, &name}) {
    if (p->empty()) continue;
    if (!s.empty()) s += "_";
    s += *p;
  }
  return s;
}

static std::string trim(const std::string& s) {
  size_t b = s.find_first_not_of(" \t\r\n"), e = s.find_last_not_of(" \t\r\n");
  return b == std::string::npos ? std::string() : s.substr(b, e - b + 1);
}

void ParamRegistry::load_files() {
  if (files_loaded_) return;
  files_loaded_ = true;
  std::vector<std::string> files;
  if (const char* env = std::getenv("PARSEC_MCA_PARAM_FILES")) {
    std::stringstream ss(env);
    std::string f;
    while (std::getline(ss, f, ':')) if (!f.empty()) files.push_back(f);
  } else {
    if (const char* home = std::getenv("HOME")) files.push_back(std::string(home) + "/.parsec/mca-params.conf");
    if (const char* pre = std::getenv("PARSEC_INSTALL_PREFIX")) files.push_back(std::string(pre) + "/etc/parsec-mca-params.conf");
  }
  // Earlier files win (user file before system file), matching the reference order.
  for (auto it = files.rbegin(); it != files.rend(); ++it) {
    std::ifstream in(*it);
    if (!in) continue;
    std::string line;
    while (std::getline(in, line)) {
      auto hash = line.find('#');
      if (hash != std::string::npos) line = line.substr(0, hash);
      auto eq = line.find('=');
      if (eq == std::string::npos) continue;
      std::string k = trim(line.substr(0, eq)), v = trim(line.substr(eq + 1));
      if (!k.empty()) file_values_[k] = {v, *it};
    }
  }
}

std::string ParamRegistry::resolve(const std::string& full, const std::string& dflt, std::string& source) {
  auto o = overrides_.find(full);
  if (o != overrides_.end()) { source = "override"; return o->second; }
  std::string env = "PARSEC_MCA_" + full;
  if (const char* v = std::getenv(env.c_str())) { source = "env"; return v; }
  load_files();
  auto f = file_values_.find(full);
  if (f != file_values_.end()) { source = "file:" + f->second.second; return f->second.first; }
  source = "default";
  return dflt;
}

static int64_t parse_int(const std::string& s, int64_t dflt) {
  if (s.empty()) return dflt;
  char* end = nullptr;
  long long v = std::strtoll(s.c_str(), &end, 0);
  if (end == s.c_str()) {
    if (s == "true" || s == "yes" || s == "on") return 1;
    if (s == "false" || s == "no" || s == "off") return 0;
    return dflt;
  }
  // size suffixes
  if (*end == 'k' || *end == 'K') v <<= 10;
  else if (*end == 'm' || *end == 'M') v <<= 20;
  else if (*end == 'g' || *end == 'G') v <<= 30;
  return v;
}

int64_t ParamRegistry::reg_int(const std::string& type, const std::string& comp, const std::string& name, const std::string& help, int64_t dflt) {
  std::lock_guard<std::mutex> g(m_);
  std::string full = join(type, comp, name);
  ParamInfo& p = params_[full];
  p.full_name = full; p.help = help; p.type = ParamType::Int; p.default_value = std::to_string(dflt);
  p.value = resolve(full, p.default_value, p.source);
  return parse_int(p.value, dflt);
}

size_t ParamRegistry::reg_sizet(const std::string& type, const std::string& comp, const std::string& name, const std::string& help, size_t dflt) {
  std::lock_guard<std::mutex> g(m_);
  std::string full = join(type, comp, name);
  ParamInfo& p = params_[full];
  p.full_name = full; p.help = help; p.type = ParamType::SizeT; p.default_value = std::to_string(dflt);
  p.value = resolve(full, p.default_value, p.source);
  return (size_t)parse_int(p.value, (int64_t)dflt);
}

std::string ParamRegistry::reg_string(const std::string& type, const std::string& comp, const std::string& name, const std::string& help, const std::string& dflt) {
  std::lock_guard<std::mutex> g(m_);
  std::string full = join(type, comp, name);
  ParamInfo& p = params_[full];
  p.full_name = full; p.help = help; p.type = ParamType::String; p.default_value = dflt;
  p.value = resolve(full, dflt, p.source);
  return p.value;
}

void ParamRegistry::set_override(const std::string& full, const std::string& value) {
  std::lock_guard<std::mutex> g(m_);
  overrides_[full] = value;
  auto it = params_.find(full);
  if (it != params_.end()) { it->second.value = value; it->second.source = "override"; }
}

void ParamRegistry::clear_override(const std::string& full) {
  std::lock_guard<std::mutex> g(m_);
  overrides_.erase(full);
  auto it = params_.find(full);
  if (it != params_.end()) it->second.value = resolve(full, it->second.default_value, it->second.source);
}

bool ParamRegistry::lookup(const std::string& full, std::string& value) {
  std::lock_guard<std::mutex> g(m_);
  auto it = params_.find(full);
  if (it != params_.end()) { value = it->second.value; return true; }
  std::string src;
  value = resolve(full, "", src);
  return src != "default";
}

std::string ParamRegistry::source(const std::string& full) {
  std::lock_guard<std::mutex> g(m_);
  auto it = params_.find(full);
  return it != params_.end() ? it->second.source : std::string();
}

std::vector<ParamInfo> ParamRegistry::dump() {
  std::lock_guard<std::mutex> g(m_);
  std::vector<ParamInfo> out;
  for (auto& kv : params_) out.push_back(kv.second);
  return out;
}

std::vector<std::string> ParamRegistry::parse_cmdline(const std::vector<std::string>& args) {
  std::vector<std::string> rest;
  for (size_t i = 0; i < args.size(); ++i) {
    if ((args[i] == "--mca" || args[i] == "-mca") && i + 2 < args.size()) {
      set_override(args[i + 1], args[i + 2]);
      i += 2;
      continue;
    }
    rest.push_back(args[i]);
  }
  return rest;
}

// ------------------------------------------------------------------ output
static std::atomic<int> g_verbosity{-1};
static std::atomic<int> g_rank{0};
static std::mutex g_out_mutex;

void output_init() {
  if (g_verbosity.load() >= 0) return;
  int v = (int)ParamRegistry::instance().reg_int("debug", "", "verbose", "Verbosity of the debug output stream", 1);
  g_verbosity.store(v);
}
int debug_verbosity() {
  int v = g_verbosity.load(std::memory_order_relaxed);
  if (v < 0) { output_init(); v = g_verbosity.load(); }
  return v;
}
int debug_rank() { return g_rank.load(); }
void set_debug_rank(int r) { g_rank.store(r); }

void outputv(int level, const char* sub, const char* fmt, va_list ap) {
  if (level > debug_verbosity()) return;
  char buf[2048];
  vsnprintf(buf, sizeof(buf), fmt, ap);
  // debug lines carry a monotonic timestamp (ms) so protocol gaps can be read off a log
  static const auto t0 = std::chrono::steady_clock::now();
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  std::lock_guard<std::mutex> g(g_out_mutex);
  if (level >= kVerbDebug) std::fprintf(stderr, "[parsec %d%s%s %.3f] %s\n", g_rank.load(), sub && *sub ? " " : "", sub ? sub : "", ms, buf);
  else std::fprintf(stderr, "[parsec %d%s%s] %s\n", g_rank.load(), sub && *sub ? " " : "", sub ? sub : "", buf);
}

void output(int level, const char* sub, const char* fmt, ...) {
  va_list ap; va_start(ap, fmt); outputv(level, sub, fmt, ap); va_end(ap);
}

void warning(const char* fmt, ...) {
  va_list ap; va_start(ap, fmt); outputv(kVerbWarn, "warning", fmt, ap); va_end(ap);
}

void fatal(const char* fmt, ...) {
  char buf[2048];
  va_list ap; va_start(ap, fmt); vsnprintf(buf, sizeof(buf), fmt, ap); va_end(ap);
  {
    std::lock_guard<std::mutex> g(g_out_mutex);
    std::fprintf(stderr, "[parsec %d FATAL] %s\n", g_rank.load(), buf);
    if (ParamRegistry::instance().reg_int("debug", "", "history_on_fatal", "Dump the debug history ring on fatal errors", 0)) {
      for (auto& s : history_dump()) std::fprintf(stderr, "  history: %s\n", s.c_str());
    }
    std::fflush(stderr);
  }
  std::abort();
}

// History ring: per-thread fixed ring, registered globally for dumps.
namespace {
constexpr int kHistLen = 256;
struct HistRing {
  char entries[kHistLen][128];
  std::atomic<uint32_t> pos{0};
};
std::mutex g_hist_m;
std::vector<HistRing*>& rings() { static std::vector<HistRing*> r; return r; }
HistRing* my_ring() {
  thread_local HistRing* r = nullptr;
  if (!r) {
    r = new HistRing();
    std::memset(r->entries, 0, sizeof(r->entries));
    std::lock_guard<std::mutex> g(g_hist_m);
    rings().push_back(r);
  }
  return r;
}
}  // namespace

void history_add(const char* fmt, ...) {
  HistRing* r = my_ring();
  uint32_t p = r->pos.fetch_add(1, std::memory_order_relaxed) % kHistLen;
  va_list ap; va_start(ap, fmt); vsnprintf(r->entries[p], sizeof(r->entries[p]), fmt, ap); va_end(ap);
}

std::vector<std::string> history_dump() {
  std::vector<std::string> out;
  std::lock_guard<std::mutex> g(g_hist_m);
  for (HistRing* r : rings()) {
    uint32_t p = r->pos.load();
    uint32_t n = p < kHistLen ? p : kHistLen;
    for (uint32_t i = 0; i < n; ++i) out.emplace_back(r->entries[(p - n + i) % kHistLen]);
  }
  return out;
}

}  // namespace parsec
