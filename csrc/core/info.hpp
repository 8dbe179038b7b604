// Info registry: named, lazily constructed per-object slots (reference
// parsec/class/info.{h,c}). A registry maps names to small ids; every object
// that carries an InfoArray (here: each HIP execution stream, each device)
// holds one slot per id, built on first use by the registered constructor and
// destroyed with the object. Used for library handles that must exist once
// per stream (e.g. a BLAS handle bound to the stream).
#pragma once

#include <atomic>
#include <functional>
#include <mutex>
#include <string>
#include <vector>

namespace parsec {

class InfoRegistry {
 public:
  using Ctor = std::function<void*(void* owner)>;
  using Dtor = std::function<void(void* elt)>;
  struct Entry {
    std::string name;
    Ctor ctor;
    Dtor dtor;
    bool live = false;
  };
  // returns the id (an existing live entry of the same name is replaced)
  int register_info(const std::string& name, Ctor ctor, Dtor dtor) {
    std::lock_guard<std::mutex> g(m_);
    for (size_t i = 0; i < e_.size(); ++i)
      if (e_[i].live && e_[i].name == name) { e_[i].ctor = std::move(ctor); e_[i].dtor = std::move(dtor); return (int)i; }
    e_.push_back({name, std::move(ctor), std::move(dtor), true});
    return (int)e_.size() - 1;
  }
  int unregister_info(int id) {
    std::lock_guard<std::mutex> g(m_);
    if (id < 0 || id >= (int)e_.size() || !e_[id].live) return -1;
    e_[id].live = false;
    return id;
  }
  int lookup(const std::string& name) const {
    std::lock_guard<std::mutex> g(m_);
    for (size_t i = 0; i < e_.size(); ++i) if (e_[i].live && e_[i].name == name) return (int)i;
    return -1;
  }
  Entry entry(int id) const {
    std::lock_guard<std::mutex> g(m_);
    return id >= 0 && id < (int)e_.size() ? e_[id] : Entry{};
  }
  int size() const {
    std::lock_guard<std::mutex> g(m_);
    return (int)e_.size();
  }

 private:
  mutable std::mutex m_;
  std::vector<Entry> e_;
};

// Per-object slots of one registry (reference parsec_info_object_array_t).
class InfoArray {
 public:
  InfoArray(InfoRegistry* reg, void* owner) : reg_(reg), owner_(owner) {}
  InfoArray(const InfoArray&) = delete;
  InfoArray& operator=(const InfoArray&) = delete;
  ~InfoArray() { clear(); }
  // slot value, constructed on first use (nullptr: no such live id / no constructor)
  void* get(int id) {
    if (void* v = peek(id)) return v;
    InfoRegistry::Entry e = reg_->entry(id);
    if (!e.live || !e.ctor) return nullptr;
    void* v = e.ctor(owner_);
    void* old = test_and_set(id, v, nullptr);
    if (old) {  // lost the race: keep the winner's object
      if (e.dtor) e.dtor(v);
      return old;
    }
    return v;
  }
  void* peek(int id) {
    std::lock_guard<std::mutex> g(m_);
    return id >= 0 && id < (int)slots_.size() ? slots_[id] : nullptr;
  }
  // set the slot to `v` when it holds `expect`; returns the previous value
  void* test_and_set(int id, void* v, void* expect) {
    std::lock_guard<std::mutex> g(m_);
    if (id < 0) return nullptr;
    if ((int)slots_.size() <= id) slots_.resize(id + 1, nullptr);
    void* cur = slots_[id];
    if (cur == expect) slots_[id] = v;
    return cur;
  }
  void* set(int id, void* v) {
    std::lock_guard<std::mutex> g(m_);
    if (id < 0) return nullptr;
    if ((int)slots_.size() <= id) slots_.resize(id + 1, nullptr);
    void* old = slots_[id];
    slots_[id] = v;
    return old;
  }
  void clear() {
    std::vector<void*> s;
    {
      std::lock_guard<std::mutex> g(m_);
      s.swap(slots_);
    }
    for (size_t i = 0; i < s.size(); ++i)
      if (s[i]) {
        InfoRegistry::Entry e = reg_->entry((int)i);
        if (e.dtor) e.dtor(s[i]);
      }
  }

 private:
  InfoRegistry* reg_;
  void* owner_;
  std::mutex m_;
  std::vector<void*> slots_;
};

// Registry of the per-GPU-execution-stream infos (reference parsec_per_stream_infos)
InfoRegistry& gpu_stream_infos();

}  // namespace parsec
