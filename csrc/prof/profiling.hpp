// Tracing / instrumentation.
//
// Parity: PBP profiling (reference profiling.h, profiling.c:473-1485 — per-stream
// event buffers, dictionary of begin/end keys with info convertors, one trace
// file per rank), PINS callback chains on 16 events (mca/pins/pins.h:26-190) with
// modules task_profiler / print_steals / alperf / iterators_checker, DOT grapher
// (parsec_prof_grapher.c:86-266), properties dictionary (dictionary.h:14-60).
// File format here is our own ("PAMDPRF2", see parsec_amd/profiling.py reader).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../core/runtime.hpp"

namespace parsec {

struct ProfEvent {
  uint16_t key;       // dictionary key (begin = 2*k, end = 2*k+1)
  uint16_t flags;     // bit0: has info
  uint32_t taskpool_id;
  uint64_t event_id;
  uint64_t timestamp; // ns since profiling start
  uint32_t info_off;  // offset in the stream's info blob
  uint32_t info_len;
};

// One event buffer per thread (or per device stream). When `events` reaches
// the buffer size (MCA profile_buffer_events) it is handed to the writer
// thread, which appends it to this stream's spill files; memory stays bounded
// and the file is assembled at fini (reference profiling.c:384-432 buffers
// flushed by a helper thread).
struct ProfilingStream {
  std::string name;
  int thread_id = 0;
  std::vector<ProfEvent> events;
  std::vector<uint8_t> info;
  uint64_t info_base = 0;       // info bytes already spilled (info_off is stream-global)
  uint64_t spilled_events = 0;  // events already handed to the writer
  std::string spill_ev, spill_info;  // spill file paths
  SpinLock lock;  // only for streams shared by several threads (devices)
  std::vector<std::pair<std::string, std::string>> infos;  // per-stream key / value pairs
};

struct DictEntry {
  std::string name;
  std::string attributes;  // e.g. "fill:#FF0000"
  std::string info_desc;   // convertor, e.g. "size{int64_t};key{uint64_t}"
  size_t info_length = 0;
};

// global enable (set when profile_filename is given)
bool profiling_enabled();
void profiling_init(Context* ctx);
void profiling_fini(Context* ctx);
void profiling_thread_init(ExecutionStream* es);
void profiling_thread_fini(ExecutionStream* es);
ProfilingStream* profiling_stream_create(const std::string& name);
// returns the key pair (begin key = 2*id, end = 2*id+1)
int profiling_add_dictionary_keyword(const std::string& name, const std::string& attributes, size_t info_length,
                                     const std::string& info_desc, int* begin_key, int* end_key);
int profiling_trace(ProfilingStream* s, int key, uint64_t event_id, uint32_t taskpool_id, const void* info, size_t info_len);
// Same with an explicit timestamp (ns on the profiling clock), e.g. GPU spans
// converted from HIP events; `s` may be shared (its lock is taken).
int profiling_trace_at(ProfilingStream* s, int key, uint64_t event_id, uint32_t taskpool_id, uint64_t timestamp, const void* info, size_t info_len);
ProfilingStream* profiling_stream_create(const std::string& name);
// Process resource usage (getrusage) as "name=value" pairs; also recorded in the
// trace header at fini and printed when runtime_report_rusage is set
// (reference parsec.c:107-145).
std::vector<std::pair<std::string, double>> profiling_rusage();
uint64_t profiling_now();
int profiling_dump(const std::string& filename);
int profiling_reset();
void profiling_add_information(const std::string& key, const std::string& value);
void profiling_start();
// ---- standalone use without a runtime context (reference profiling.h:133-461:
// init / dbp_start / stream_init / trace_flags / dbp_dump / fini from any
// number of application threads, one stream each)
int profiling_standalone_init(int rank);
int profiling_dbp_start(const std::string& basefile, const std::string& hr_id);
int profiling_dbp_dump();  // <basefile>-<rank>.prof
int profiling_standalone_fini();
void profiling_stream_add_information(ProfilingStream* s, const std::string& key, const std::string& value);
int profiling_dictionary_flush();
size_t profiling_key_info_length(int key);  // info bytes of a begin / end key
void profiling_set_recording(bool on);      // parsec_profiling_enable / disable
const char* profiling_last_error();

// PINS
void pins_init(Context* ctx);
void pins_fini(Context* ctx);
using PinsCallback = std::function<void(ExecutionStream*, int event, Task*)>;
int pins_register_callback(int event, PinsCallback cb);
std::vector<std::string> pins_modules_available();
// counters exposed by the alperf / print_steals modules
std::vector<std::pair<std::string, int64_t>> pins_counters();

// ptg_to_dtd PINS module (ptg_to_dtd.cpp)
void ptg_to_dtd_enable(bool on);
bool ptg_to_dtd_enabled();
int64_t ptg_to_dtd_redirected();
void ptg_to_dtd_taskpool_init(Context* ctx, Taskpool* tp);

// DOT grapher
void grapher_init(Context* ctx);
void grapher_task(ExecutionStream* es, Task* t);
void grapher_dep(ExecutionStream* es, const Task* from, const TaskClass* to_tc, const int32_t* to_locals, int nb_locals, int from_flow, int to_flow);
void grapher_fini(Context* ctx);

// Properties dictionary (live counters readable by tools)
void properties_set(const std::string& name, double value);
void properties_publisher_start(Context* ctx);
void properties_publisher_stop();
std::vector<std::pair<std::string, double>> properties_snapshot();
int properties_dump_shm(const std::string& shm_name);

}  // namespace parsec
