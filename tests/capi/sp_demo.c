/* Standalone profiling from C, no runtime context (port of the reference's
 * tests/profiling-standalone/sp-demo.c:72-195): NB_THREADS threads each open
 * their own stream, add a per-stream key / value, and trace EVENTS_PER_THREAD
 * begin / end pairs of two event types, the second one carrying an info
 * structure {int i; double d}; the main thread sets time 0 once every stream
 * exists, then dumps <base>-0.prof. With "perf" as argv[1] it times
 * argv[3] (default 1M) begin / end pairs per thread instead (sp-perf.c) and
 * prints ns / event. Usage: sp_demo demo|perf [base] [pairs].
 * Differences: no MPI (the reference initialises it only for its OTF2
 * backend); the file name is <base>-<rank>.prof. */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "parsec.h"

#define NB_THREADS 4
#define EVENTS_PER_THREAD 10

typedef struct {
  pthread_t pthread_id;
  int thread_index;
  parsec_profiling_stream_t* prof;
  unsigned seed;
} per_thread_info_t;

typedef struct {
  int i;
  double d;
} event_b_info_t;

static pthread_barrier_t barrier;
static int event_a_startkey, event_a_endkey;
static int event_b_startkey, event_b_endkey;
static int perf_mode = 0;
static long perf_events = 1000000;

static void* run_thread(void* arg) {
  per_thread_info_t* ti = (per_thread_info_t*)arg;
  ti->prof = parsec_profiling_stream_init(4096, "This is the name of thread %d", ti->thread_index);
  pthread_barrier_wait(&barrier); /* every stream exists: main sets time 0 */
  parsec_profiling_stream_add_information(ti->prof, "This is a thread-specific information key", "This is the corresponding value");
  pthread_barrier_wait(&barrier); /* time 0 is set */
  if (perf_mode) {
    for (long i = 0; i < perf_events; i++) {
      parsec_profiling_trace_flags(ti->prof, event_a_startkey, (uint64_t)i, PROFILE_OBJECT_ID_NULL, NULL, 0);
      parsec_profiling_trace_flags(ti->prof, event_a_endkey, (uint64_t)i, PROFILE_OBJECT_ID_NULL, NULL, 0);
    }
    return NULL;
  }
  for (int i = 0; i < EVENTS_PER_THREAD; i++) {
    if (rand_r(&ti->seed) % 2 == 0) {
      parsec_profiling_trace_flags(ti->prof, event_a_startkey, (uint64_t)i, PROFILE_OBJECT_ID_NULL, NULL, 0);
      usleep(rand_r(&ti->seed) % 300);
      parsec_profiling_trace_flags(ti->prof, event_a_endkey, (uint64_t)i, PROFILE_OBJECT_ID_NULL, NULL, 0);
    } else {
      event_b_info_t info;
      info.i = i;
      info.d = (double)ti->thread_index;
      parsec_profiling_trace_flags(ti->prof, event_b_startkey, (uint64_t)i, PROFILE_OBJECT_ID_NULL, NULL, 0);
      usleep(rand_r(&ti->seed) % 300);
      parsec_profiling_trace_flags(ti->prof, event_b_endkey, (uint64_t)i, PROFILE_OBJECT_ID_NULL, &info, PARSEC_PROFILING_EVENT_HAS_INFO);
    }
  }
  return NULL;
}

int main(int argc, char* argv[]) {
  per_thread_info_t thread_info[NB_THREADS];
  const char* base = argc > 2 ? argv[2] : "sp";
  perf_mode = argc > 1 && strcmp(argv[1], "perf") == 0;
  if (argc > 3) perf_events = atol(argv[3]);
  if (parsec_profiling_init(0) != PARSEC_SUCCESS) return 1;
  if (parsec_profiling_dbp_start(base, "Demonstration of basic PaRSEC profiling system") != PARSEC_SUCCESS) {
    fprintf(stderr, "dbp_start: %s\n", parsec_profiling_strerror());
    return 1;
  }
  parsec_profiling_add_dictionary_keyword("Event A", "#FF0000", 0, NULL, &event_a_startkey, &event_a_endkey);
  parsec_profiling_add_dictionary_keyword("Event B", "#0000FF", sizeof(event_b_info_t), "i{int32_t};d{double}", &event_b_startkey, &event_b_endkey);
  parsec_profiling_add_information("This is a global information key", "This is the global information value");

  pthread_barrier_init(&barrier, NULL, NB_THREADS + 1);
  for (int i = 0; i < NB_THREADS; i++) {
    thread_info[i].thread_index = i;
    thread_info[i].seed = 1234u + (unsigned)i;
    pthread_create(&thread_info[i].pthread_id, NULL, run_thread, &thread_info[i]);
  }
  pthread_barrier_wait(&barrier);
  parsec_profiling_start();
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  pthread_barrier_wait(&barrier);
  for (int i = 0; i < NB_THREADS; i++) pthread_join(thread_info[i].pthread_id, NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  if (perf_mode) {
    const double ns = (t1.tv_sec - t0.tv_sec) * 1e9 + (t1.tv_nsec - t0.tv_nsec);
    printf("sp-perf: %d threads x %ld event pairs: %.1f ns per event per thread\n", NB_THREADS, perf_events, ns / (2.0 * perf_events));
  }
  if (parsec_profiling_dbp_dump() != PARSEC_SUCCESS) {
    fprintf(stderr, "dbp_dump: %s\n", parsec_profiling_strerror());
    return 1;
  }
  parsec_profiling_fini();
  pthread_barrier_destroy(&barrier);
  printf("sp-demo done\n");
  return 0;
}
