// Futures: one-shot values that a producer sets and consumers wait for.
//
// Reference: parsec/class/parsec_future.{h,c} and parsec_datacopy_future.c.
// Three kinds, same roles as the reference:
//   BaseFuture      set once, get blocks until set, optional fulfil callback
//                   run by the setter (parsec_future.c:40-120)
//   CountableFuture ready after `count` set() calls (parsec_future.c:122-180)
//   DatacopyFuture  lazily produced value: the first get_or_trigger() runs
//                   the fulfil callback, concurrent callers wait for it; a
//                   request that does not match this future's spec is served
//                   by a nested future (created on demand) so that every
//                   distinct spec is produced exactly once
//                   (parsec_datacopy_future.c:30-260)
// The reshape engine keys one DatacopyFuture per source copy and uses the
// target datatype as the spec: successors asking for the same layout share
// one reshaped copy (parsec_reshape.c:29-771).
//
// Written for this runtime: std::atomic status + SpinLock, waiting with a
// bounded spin then yield (futures are resolved by runtime threads that are
// always making progress).
#pragma once

#include <atomic>
#include <functional>
#include <thread>
#include <vector>

#include "core/base.hpp"

namespace parsec {

enum FutureStatus : uint8_t { FUTURE_INIT = 0x1, FUTURE_TRIGGERED = 0x2, FUTURE_COMPLETED = 0x4 };

class BaseFuture {
 public:
  using Fulfill = std::function<void(BaseFuture*)>;
  explicit BaseFuture(Fulfill on_set = nullptr) : on_set_(std::move(on_set)) {}
  virtual ~BaseFuture() = default;
  virtual bool is_ready() const { return status_.load(std::memory_order_acquire) & FUTURE_COMPLETED; }
  // publish the value; the fulfil callback (if any) runs on the setter
  virtual void set(void* v) {
    value_ = v;
    status_.fetch_or(FUTURE_COMPLETED, std::memory_order_acq_rel);
    if (on_set_) on_set_(this);
  }
  void* get() const {
    wait_ready();
    return value_;
  }
  void* peek() const { return is_ready() ? value_ : nullptr; }
  uint8_t status() const { return status_.load(std::memory_order_acquire); }

 protected:
  void wait_ready() const {
    for (int spins = 0; !is_ready(); ++spins) {
      if (spins < 256) PARSEC_CPU_RELAX();
      else std::this_thread::yield();
    }
  }
  std::atomic<uint8_t> status_{FUTURE_INIT};
  void* value_ = nullptr;
  Fulfill on_set_;
};

class CountableFuture : public BaseFuture {
 public:
  explicit CountableFuture(int32_t count, Fulfill on_ready = nullptr) : BaseFuture(std::move(on_ready)), count_(count) {
    if (count <= 0) BaseFuture::set(nullptr);
  }
  // each call counts down; the value passed with the last one is kept
  void set(void* v) override {
    if (count_.fetch_sub(1, std::memory_order_acq_rel) == 1) BaseFuture::set(v);
  }
  int32_t remaining() const { return count_.load(std::memory_order_acquire); }

 private:
  std::atomic<int32_t> count_;
};

class DatacopyFuture : public BaseFuture {
 public:
  // produce(in, spec) returns the value for `spec`; match(spec_a, spec_b)
  // says whether two specs describe the same value; cleanup(value) releases a
  // produced value when the future dies.
  using Produce = std::function<void*(void* in, const void* spec)>;
  using Match = std::function<bool(const void* a, const void* b)>;
  using Cleanup = std::function<void(void* value)>;

  DatacopyFuture(void* in, const void* spec, Produce produce, Match match, Cleanup cleanup, bool nested_enable = true)
      : in_(in), spec_(spec), produce_(std::move(produce)), match_(std::move(match)), cleanup_(std::move(cleanup)), nested_enable_(nested_enable) {}
  ~DatacopyFuture() override {
    if (is_ready() && cleanup_) cleanup_(value_);
    for (DatacopyFuture* n : nested_) delete n;
  }
  const void* spec() const { return spec_; }

  // The value for `spec` (this future's own when spec matches it, else a
  // nested one), produced by exactly one caller.
  void* get_or_trigger(const void* spec) {
    // a root future created without a spec only dispatches to nested ones
    if (spec_ ? match_(spec_, spec) : !spec) return trigger_self();
    if (!nested_enable_) return nullptr;
    DatacopyFuture* n = nullptr;
    {
      std::lock_guard<SpinLock> g(lock_);
      for (DatacopyFuture* c : nested_)
        if (match_(c->spec_, spec)) { n = c; break; }
      if (!n) {
        // the nested future owns no spec storage: callers pass specs that
        // live as long as the taskpool (arena datatypes)
        n = new DatacopyFuture(in_, spec, produce_, match_, cleanup_, false);
        nested_.push_back(n);
      }
    }
    return n->trigger_self();
  }
  size_t nested_count() {
    std::lock_guard<SpinLock> g(lock_);
    return nested_.size();
  }

 private:
  void* trigger_self() {
    uint8_t s = status_.fetch_or(FUTURE_TRIGGERED, std::memory_order_acq_rel);
    if (!(s & FUTURE_TRIGGERED)) set(produce_(in_, spec_));  // first caller produces
    return get();
  }
  void* in_;
  const void* spec_;
  Produce produce_;
  Match match_;
  Cleanup cleanup_;
  bool nested_enable_;
  SpinLock lock_;
  std::vector<DatacopyFuture*> nested_;
};

}  // namespace parsec
