// Minimal MPI (include/mpi/mpi.h) over this runtime's communication engine,
// so programs written against PaRSEC + MPI -- the reference's multi-process
// tests -- build and run unmodified under parsec_amd.launch. Reference: the
// MPI calls of those programs and of the comm bring-up they pair with
// (remote_dep_mpi.c:250-338 requires MPI_THREAD_SERIALIZED or better; the
// runtime here shares the engine the program initialized, as PaRSEC shares the
// application's MPI).
//
// Every collective is gather-to-first-member + broadcast over active messages
// on TAG_MPI_SHIM: member i sends (communicator id, sequence number, its
// contribution) to member 0, which combines in member order and sends the
// result back. Messages land in a mailbox keyed by (communicator, sequence,
// kind, member); the calling thread blocks on a condition variable while the
// engine's comm thread delivers. Communicators created by split / dup get an id
// derived from the parent's id, the parent's sequence number and the colour,
// identical on every member without extra traffic.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <functional>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <unistd.h>
#include <vector>

#include "../comm/comm.hpp"
#include "../core/mca.hpp"
#include "../../include/mpi/mpi.h"

namespace parsec {
bool& comm_owned_by_mpi();
}

namespace {
using namespace parsec;

struct Comm {
  uint64_t gid;
  std::vector<int> members;  // world ranks, in communicator rank order
  int me = -1;               // my rank in the communicator
  uint64_t seq = 0;          // collectives issued on it
  bool alive = true;
};

struct Shim {
  std::mutex m;
  std::condition_variable cv;
  std::vector<Comm> comms;  // handle = index; 0 WORLD, 1 SELF
  // (gid, seq, kind, member) -> payload; kind 0 contribution, 1 result
  std::map<std::tuple<uint64_t, uint64_t, int, int>, std::vector<char>> box;
  bool init = false, fini = false, own_engine = false;
};
Shim& S() {
  static Shim* s = new Shim();
  return *s;
}

struct Hdr {
  uint64_t gid, seq;
  int32_t kind, member;
};

size_t type_size(MPI_Datatype t) {
  switch (t) {
    case MPI_CHAR: case MPI_BYTE: return 1;
    case MPI_SHORT: case MPI_UNSIGNED_SHORT: return 2;
    case MPI_INT: case MPI_UNSIGNED: case MPI_FLOAT: return 4;
    case MPI_LONG: case MPI_UNSIGNED_LONG: case MPI_LONG_LONG: case MPI_UNSIGNED_LONG_LONG: case MPI_DOUBLE: return 8;
    case MPI_2INT: return 8;
    case MPI_DOUBLE_INT: return 16;  // {double, int} padded
    case MPI_LONG_INT: return 16;
    default: return 0;
  }
}

template <class T>
void red(T* io, const T* in, int n, MPI_Op op) {
  for (int i = 0; i < n; ++i) {
    switch (op) {
      case MPI_SUM: io[i] = io[i] + in[i]; break;
      case MPI_PROD: io[i] = io[i] * in[i]; break;
      case MPI_MAX: io[i] = in[i] > io[i] ? in[i] : io[i]; break;
      case MPI_MIN: io[i] = in[i] < io[i] ? in[i] : io[i]; break;
      case MPI_LAND: io[i] = (io[i] != T(0)) && (in[i] != T(0)); break;
      case MPI_LOR: io[i] = (io[i] != T(0)) || (in[i] != T(0)); break;
      default: fatal("MPI shim: reduction %d not supported on this type", op);
    }
  }
}
template <class T>
void red_bits(T* io, const T* in, int n, MPI_Op op) {
  if (op == MPI_BAND) { for (int i = 0; i < n; ++i) io[i] &= in[i]; return; }
  if (op == MPI_BOR) { for (int i = 0; i < n; ++i) io[i] |= in[i]; return; }
  red(io, in, n, op);
}
template <class V>
void red_loc(char* io, const char* in, int n, MPI_Op op, size_t stride) {
  // {value, int index}: MAXLOC / MINLOC keep the extreme value, lowest index on ties
  for (int i = 0; i < n; ++i) {
    V a, b;
    int ia, ib;
    std::memcpy(&a, io + i * stride, sizeof(V));
    std::memcpy(&b, in + i * stride, sizeof(V));
    std::memcpy(&ia, io + i * stride + sizeof(V), sizeof(int));
    std::memcpy(&ib, in + i * stride + sizeof(V), sizeof(int));
    const bool take = op == MPI_MAXLOC ? (b > a || (b == a && ib < ia)) : (b < a || (b == a && ib < ia));
    if (op != MPI_MAXLOC && op != MPI_MINLOC) fatal("MPI shim: pair types support MAXLOC / MINLOC only");
    if (take) std::memcpy(io + i * stride, in + i * stride, stride);
  }
}
void reduce_into(char* io, const char* in, int count, MPI_Datatype t, MPI_Op op) {
  switch (t) {
    case MPI_CHAR: red_bits((signed char*)io, (const signed char*)in, count, op); break;
    case MPI_BYTE: red_bits((unsigned char*)io, (const unsigned char*)in, count, op); break;
    case MPI_SHORT: red_bits((short*)io, (const short*)in, count, op); break;
    case MPI_UNSIGNED_SHORT: red_bits((unsigned short*)io, (const unsigned short*)in, count, op); break;
    case MPI_INT: red_bits((int*)io, (const int*)in, count, op); break;
    case MPI_UNSIGNED: red_bits((unsigned*)io, (const unsigned*)in, count, op); break;
    case MPI_LONG: red_bits((long*)io, (const long*)in, count, op); break;
    case MPI_UNSIGNED_LONG: red_bits((unsigned long*)io, (const unsigned long*)in, count, op); break;
    case MPI_LONG_LONG: red_bits((long long*)io, (const long long*)in, count, op); break;
    case MPI_UNSIGNED_LONG_LONG: red_bits((unsigned long long*)io, (const unsigned long long*)in, count, op); break;
    case MPI_FLOAT: red((float*)io, (const float*)in, count, op); break;
    case MPI_DOUBLE: red((double*)io, (const double*)in, count, op); break;
    case MPI_2INT: red_loc<int>(io, in, count, op, 8); break;
    case MPI_DOUBLE_INT: red_loc<double>(io, in, count, op, 16); break;
    case MPI_LONG_INT: red_loc<long>(io, in, count, op, 16); break;
    default: fatal("MPI shim: datatype %d not supported", t);
  }
}

Comm& comm_of(MPI_Comm c) {
  Shim& s = S();
  if (!s.init) fatal("MPI shim: MPI_Init was not called");
  if (c < 0 || c >= (int)s.comms.size() || !s.comms[(size_t)c].alive) fatal("MPI shim: invalid communicator %d", c);
  return s.comms[(size_t)c];
}

void on_msg(int src, int, const void* msg, size_t len) {
  (void)src;
  Hdr h;
  std::memcpy(&h, msg, sizeof(h));
  std::vector<char> payload(static_cast<const char*>(msg) + sizeof(h), static_cast<const char*>(msg) + len);
  Shim& s = S();
  {
    std::lock_guard<std::mutex> g(s.m);
    s.box[std::make_tuple(h.gid, h.seq, (int)h.kind, (int)h.member)] = std::move(payload);
  }
  s.cv.notify_all();
}

void send_to(int world_rank, const Hdr& h, const void* data, size_t n) {
  std::vector<char> m(sizeof(h) + n);
  std::memcpy(m.data(), &h, sizeof(h));
  if (n) std::memcpy(m.data() + sizeof(h), data, n);
  if (comm_engine()->send_am(TAG_MPI_SHIM, world_rank, m.data(), m.size()) != 0) fatal("MPI shim: send to rank %d failed", world_rank);
}

std::vector<char> take(uint64_t gid, uint64_t seq, int kind, int member) {
  Shim& s = S();
  std::unique_lock<std::mutex> g(s.m);
  const auto key = std::make_tuple(gid, seq, kind, member);
  s.cv.wait(g, [&] { return s.box.count(key) != 0; });
  std::vector<char> v = std::move(s.box[key]);
  s.box.erase(key);
  return v;
}

// The collective core: every member contributes `mine`; the first member gets
// all contributions (member order) and computes the result with `combine`; every
// member returns that result.
std::vector<char> collective(Comm& c, const std::vector<char>& mine, const std::function<std::vector<char>(std::vector<std::vector<char>>&)>& combine) {
  const uint64_t seq = c.seq++;
  const int n = (int)c.members.size();
  if (n == 1) {
    std::vector<std::vector<char>> all{mine};
    return combine(all);
  }
  if (c.me != 0) {
    send_to(c.members[0], Hdr{c.gid, seq, 0, c.me}, mine.data(), mine.size());
    return take(c.gid, seq, 1, 0);
  }
  std::vector<std::vector<char>> all((size_t)n);
  all[0] = mine;
  for (int i = 1; i < n; ++i) all[(size_t)i] = take(c.gid, seq, 0, i);
  std::vector<char> res = combine(all);
  for (int i = 1; i < n; ++i) send_to(c.members[(size_t)i], Hdr{c.gid, seq, 1, 0}, res.data(), res.size());
  return res;
}

std::vector<char> bytes_of(const void* p, size_t n) {
  const char* b = static_cast<const char*>(p);
  return std::vector<char>(b, b + n);
}

uint64_t mix(uint64_t a, uint64_t b) {
  uint64_t x = a * 0x9E3779B97F4A7C15ull ^ (b + 0x632BE59BD9B4E019ull + (a << 6) + (a >> 2));
  x ^= x >> 31;
  x *= 0xBF58476D1CE4E5B9ull;
  return x ^ (x >> 29);
}
}  // namespace

namespace parsec {
bool& comm_owned_by_mpi() {
  static bool v = false;
  return v;
}
}  // namespace parsec

extern "C" {

int MPI_Init_thread(int* argc, char*** argv, int required, int* provided) {
  (void)argc;
  (void)argv;
  (void)required;
  Shim& s = S();
  if (s.init) fatal("MPI shim: MPI_Init called twice");
  int rank = 0, size = 1;
  const char* r = getenv("PARSEC_COMM_RANK");
  const char* z = getenv("PARSEC_COMM_SIZE");
  if (!r) r = getenv("RANK");
  if (!z) z = getenv("WORLD_SIZE");
  if (r && z) { rank = atoi(r); size = atoi(z); }
  if (size > 1 && comm_size() <= 1) {
    const char* job = getenv("PARSEC_COMM_JOB");
    const char* g = getenv("PARSEC_COMM_GPU");
    if (comm_init(rank, size, job ? job : (getenv("MASTER_PORT") ? getenv("MASTER_PORT") : "mpi"), g ? atoi(g) : -1) != 0) fatal("MPI shim: communication engine start-up failed");
    s.own_engine = true;
    comm_owned_by_mpi() = true;  // parsec_fini leaves the engine to MPI_Finalize
  }
  if (size > 1) comm_engine()->tag_register(TAG_MPI_SHIM, on_msg);
  Comm world{0x57u, {}, rank};
  for (int i = 0; i < size; ++i) world.members.push_back(i);
  Comm self{mix(0x5e1fu, (uint64_t)rank), {rank}, 0};
  s.comms = {world, self};
  s.init = true;
  if (provided) *provided = MPI_THREAD_MULTIPLE;
  return MPI_SUCCESS;
}
int MPI_Init(int* argc, char*** argv) {
  int p;
  return MPI_Init_thread(argc, argv, MPI_THREAD_SINGLE, &p);
}
int MPI_Initialized(int* flag) {
  *flag = S().init ? 1 : 0;
  return MPI_SUCCESS;
}
int MPI_Finalized(int* flag) {
  *flag = S().fini ? 1 : 0;
  return MPI_SUCCESS;
}
int MPI_Query_thread(int* provided) {
  *provided = MPI_THREAD_MULTIPLE;
  return MPI_SUCCESS;
}
int MPI_Finalize(void) {
  Shim& s = S();
  if (!s.init || s.fini) return MPI_SUCCESS;
  MPI_Barrier(MPI_COMM_WORLD);
  s.fini = true;
  if (s.own_engine) {
    comm_owned_by_mpi() = false;
    comm_fini();
  }
  return MPI_SUCCESS;
}
int MPI_Abort(MPI_Comm comm, int errorcode) {
  (void)comm;
  std::fprintf(stderr, "MPI_Abort(%d) on rank %d\n", errorcode, comm_rank());
  std::fflush(stderr);
  _exit(errorcode ? errorcode : 1);
}
int MPI_Comm_size(MPI_Comm comm, int* size) {
  *size = (int)comm_of(comm).members.size();
  return MPI_SUCCESS;
}
int MPI_Comm_rank(MPI_Comm comm, int* rank) {
  *rank = comm_of(comm).me;
  return MPI_SUCCESS;
}
int MPI_Comm_split(MPI_Comm comm, int color, int key, MPI_Comm* newcomm) {
  Comm& c = comm_of(comm);
  const uint64_t seq = c.seq;  // the split's sequence number names the new communicators
  const int mine[3] = {color, key, c.me};
  auto all = collective(c, bytes_of(mine, sizeof(mine)), [](std::vector<std::vector<char>>& v) {
    std::vector<char> out;
    for (auto& x : v) out.insert(out.end(), x.begin(), x.end());
    return out;
  });
  const Comm parent = c;  // (the table may grow below)
  if (color == MPI_UNDEFINED) {
    *newcomm = MPI_COMM_NULL;
    return MPI_SUCCESS;
  }
  std::vector<std::tuple<int, int, int>> group;  // (key, parent rank, world rank)
  for (size_t i = 0; i < parent.members.size(); ++i) {
    int e[3];
    std::memcpy(e, all.data() + i * sizeof(e), sizeof(e));
    if (e[0] == color) group.emplace_back(e[1], e[2], parent.members[(size_t)e[2]]);
  }
  std::sort(group.begin(), group.end());
  Comm n{mix(mix(parent.gid, seq), (uint64_t)(uint32_t)color), {}, -1};
  for (auto& [k, pr, wr] : group) {
    if (pr == parent.me) n.me = (int)n.members.size();
    n.members.push_back(wr);
  }
  Shim& s = S();
  std::lock_guard<std::mutex> g(s.m);
  s.comms.push_back(n);
  *newcomm = (MPI_Comm)(s.comms.size() - 1);
  return MPI_SUCCESS;
}
int MPI_Comm_dup(MPI_Comm comm, MPI_Comm* newcomm) {
  return MPI_Comm_split(comm, 0, comm_of(comm).me, newcomm);
}
int MPI_Comm_free(MPI_Comm* comm) {
  if (!comm || *comm == MPI_COMM_NULL) return MPI_SUCCESS;
  if (*comm == MPI_COMM_WORLD || *comm == MPI_COMM_SELF) fatal("MPI shim: freeing a predefined communicator");
  comm_of(*comm).alive = false;
  *comm = MPI_COMM_NULL;
  return MPI_SUCCESS;
}
int MPI_Barrier(MPI_Comm comm) {
  collective(comm_of(comm), {}, [](std::vector<std::vector<char>>&) { return std::vector<char>(); });
  return MPI_SUCCESS;
}
int MPI_Bcast(void* buffer, int count, MPI_Datatype datatype, int root, MPI_Comm comm) {
  Comm& c = comm_of(comm);
  const size_t n = type_size(datatype) * (size_t)count;
  auto res = collective(c, c.me == root ? bytes_of(buffer, n) : std::vector<char>(), [root](std::vector<std::vector<char>>& v) { return v[(size_t)root]; });
  if (c.me != root) std::memcpy(buffer, res.data(), n);
  return MPI_SUCCESS;
}
int MPI_Allreduce(const void* sendbuf, void* recvbuf, int count, MPI_Datatype datatype, MPI_Op op, MPI_Comm comm) {
  Comm& c = comm_of(comm);
  const size_t n = type_size(datatype) * (size_t)count;
  if (!n && count) fatal("MPI shim: datatype %d not supported", datatype);
  auto res = collective(c, bytes_of(sendbuf == MPI_IN_PLACE ? recvbuf : sendbuf, n), [=](std::vector<std::vector<char>>& v) {
    std::vector<char> acc = v[0];
    for (size_t i = 1; i < v.size(); ++i) reduce_into(acc.data(), v[i].data(), count, datatype, op);
    return acc;
  });
  std::memcpy(recvbuf, res.data(), n);
  return MPI_SUCCESS;
}
int MPI_Reduce(const void* sendbuf, void* recvbuf, int count, MPI_Datatype datatype, MPI_Op op, int root, MPI_Comm comm) {
  Comm& c = comm_of(comm);
  const size_t n = type_size(datatype) * (size_t)count;
  std::vector<char> tmp(n);
  const void* in = sendbuf == MPI_IN_PLACE ? recvbuf : sendbuf;
  MPI_Allreduce(in, tmp.data(), count, datatype, op, comm);
  if (c.me == root) std::memcpy(recvbuf, tmp.data(), n);
  return MPI_SUCCESS;
}
int MPI_Allgather(const void* sendbuf, int sendcount, MPI_Datatype sendtype, void* recvbuf, int recvcount, MPI_Datatype recvtype, MPI_Comm comm) {
  Comm& c = comm_of(comm);
  const size_t rn = type_size(recvtype) * (size_t)recvcount;
  const void* in = sendbuf == MPI_IN_PLACE ? static_cast<char*>(recvbuf) + rn * (size_t)c.me : sendbuf;
  const size_t sn = sendbuf == MPI_IN_PLACE ? rn : type_size(sendtype) * (size_t)sendcount;
  if (sn != rn) fatal("MPI shim: allgather send / receive sizes differ");
  auto res = collective(c, bytes_of(in, sn), [](std::vector<std::vector<char>>& v) {
    std::vector<char> out;
    for (auto& x : v) out.insert(out.end(), x.begin(), x.end());
    return out;
  });
  std::memcpy(recvbuf, res.data(), res.size());
  return MPI_SUCCESS;
}
int MPI_Type_size(MPI_Datatype datatype, int* size) {
  *size = (int)type_size(datatype);
  return *size ? MPI_SUCCESS : MPI_ERR_OTHER;
}
int MPI_Get_processor_name(char* name, int* resultlen) {
  if (gethostname(name, MPI_MAX_PROCESSOR_NAME) != 0) std::strcpy(name, "localhost");
  name[MPI_MAX_PROCESSOR_NAME - 1] = 0;
  *resultlen = (int)std::strlen(name);
  return MPI_SUCCESS;
}
double MPI_Wtime(void) {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // extern "C"
