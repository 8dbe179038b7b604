// Configuration ("MCA parameters") and output/debug services.
//
// Parity: reference utils/mca_param.c (typed params; lookup order
// override > env PARSEC_MCA_<name> > param files > default, :95,162-231,1582-1649),
// utils/output.c + utils/debug.c (verbosity streams, history ring dumped on fatal,
// debug.c:177-), cmd-line `--mca name value` (parsec.c:417-463).
#pragma once
#include <cstdarg>
#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace parsec {

enum class ParamType { Int, SizeT, String };

struct ParamInfo {
  std::string full_name;  // "<type>_<component>_<name>" with empty parts dropped
  std::string help;
  ParamType type;
  std::string default_value;
  std::string value;   // resolved
  std::string source;  // "default" | "file:<path>" | "env" | "override"
};

class ParamRegistry {
 public:
  static ParamRegistry& instance();
  // Register (idempotent) and return the resolved value.
  int64_t reg_int(const std::string& type, const std::string& comp, const std::string& name, const std::string& help, int64_t dflt);
  size_t reg_sizet(const std::string& type, const std::string& comp, const std::string& name, const std::string& help, size_t dflt);
  std::string reg_string(const std::string& type, const std::string& comp, const std::string& name, const std::string& help, const std::string& dflt);
  // Explicit overrides: `--mca name value` or API.
  void set_override(const std::string& full_name, const std::string& value);
  void clear_override(const std::string& full_name);
  bool lookup(const std::string& full_name, std::string& value);
  // where a registered parameter's value came from ("default", "env", ...; "" if unknown)
  std::string source(const std::string& full_name);
  std::vector<ParamInfo> dump();
  void load_files();  // $HOME/.parsec/mca-params.conf, $PARSEC_MCA_PARAM_FILES
  // Parse argv: consumes "--mca k v" and "-mca k v" pairs, returns remaining args.
  std::vector<std::string> parse_cmdline(const std::vector<std::string>& args);
  static std::string join(const std::string& type, const std::string& comp, const std::string& name);

 private:
  std::string resolve(const std::string& full, const std::string& dflt, std::string& source);
  std::mutex m_;
  std::map<std::string, ParamInfo> params_;
  std::map<std::string, std::string> overrides_;
  std::map<std::string, std::pair<std::string, std::string>> file_values_;  // name -> (value, path)
  bool files_loaded_ = false;
};

// ------------------------------------------------------------------ output
enum : int { kVerbNone = 0, kVerbWarn = 1, kVerbInfo = 2, kVerbDebug = 10, kVerbNoisier = 20 };

void output_init();
int debug_verbosity();
int debug_rank();
void set_debug_rank(int r);
void outputv(int level, const char* subsystem, const char* fmt, va_list ap);
void output(int level, const char* subsystem, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
[[noreturn]] void fatal(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
void warning(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
// Per-thread lock-free history ring (reference PARSEC_DEBUG_HISTORY).
void history_add(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
std::vector<std::string> history_dump();

#define PARSEC_DEBUG(level, sub, ...) \
  do { if (::parsec::debug_verbosity() >= (level)) ::parsec::output((level), (sub), __VA_ARGS__); } while (0)

}  // namespace parsec
