// Per-shard bulk memory on transparent huge pages.  A caller shard touches
// hundreds of MB of fresh memory (its reads' bases and qualities, the
// window's pileup arrays); on 4 KiB pages that is ~10^5 page faults per shard,
// and with 32 shard threads in one process the faults and the allocator's
// heap growth serialize on the process's memory-map lock (the 31 Mbp htc
// profile: 2.3 M minor faults, more system than user time).  Anonymous
// mappings advised MADV_HUGEPAGE fault 2 MiB at a time and arrive zeroed.
#pragma once

#include <sys/mman.h>

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <new>
#include <utility>
#include <vector>

namespace fcsg {

// One zero-filled anonymous mapping of at least `bytes`.
class HugeBuf {
 public:
  static constexpr size_t kHuge = size_t(2) << 20;
  HugeBuf() = default;
  explicit HugeBuf(size_t bytes) {
    if (bytes == 0) return;
    len_ = (bytes + kHuge - 1) / kHuge * kHuge;
    void* p = ::mmap(nullptr, len_, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) {
      len_ = 0;
      throw std::bad_alloc();
    }
    ::madvise(p, len_, MADV_HUGEPAGE);  // advisory: 4 KiB pages when THP is off
    p_ = static_cast<uint8_t*>(p);
  }
  ~HugeBuf() { release(); }
  HugeBuf(const HugeBuf&) = delete;
  HugeBuf& operator=(const HugeBuf&) = delete;
  HugeBuf(HugeBuf&& o) noexcept : p_(std::exchange(o.p_, nullptr)), len_(std::exchange(o.len_, 0)) {}
  HugeBuf& operator=(HugeBuf&& o) noexcept {
    if (this != &o) {
      release();
      p_ = std::exchange(o.p_, nullptr);
      len_ = std::exchange(o.len_, 0);
    }
    return *this;
  }
  uint8_t* data() const { return p_; }
  size_t capacity() const { return len_; }

 private:
  void release() {
    if (p_) ::munmap(p_, len_);
    p_ = nullptr;
    len_ = 0;
  }
  uint8_t* p_ = nullptr;
  size_t len_ = 0;
};

// A fixed-size zero-initialised array of trivially copyable T on a HugeBuf.
template <typename T>
class HugeArray {
 public:
  HugeArray() = default;
  explicit HugeArray(size_t n) : buf_(n * sizeof(T)), n_(n) {}
  T& operator[](size_t i) { return data()[i]; }
  const T& operator[](size_t i) const { return data()[i]; }
  T* data() { return reinterpret_cast<T*>(buf_.data()); }
  const T* data() const { return reinterpret_cast<const T*>(buf_.data()); }
  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }

 private:
  HugeBuf buf_;
  size_t n_ = 0;
};

// A growable array of trivially copyable T on a HugeBuf (the subset of
// std::vector the caller uses); growth doubles and copies.
template <typename T>
class HugeVec {
 public:
  T* begin() { return data(); }
  T* end() { return data() + n_; }
  const T* begin() const { return data(); }
  const T* end() const { return data() + n_; }
  T* data() { return reinterpret_cast<T*>(buf_.data()); }
  const T* data() const { return reinterpret_cast<const T*>(buf_.data()); }
  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  T& operator[](size_t i) { return data()[i]; }
  const T& operator[](size_t i) const { return data()[i]; }
  void clear() { n_ = 0; }
  void reserve(size_t cap) {
    if (cap * sizeof(T) <= buf_.capacity()) return;
    HugeBuf nb(cap * sizeof(T));
    if (n_) std::memcpy(nb.data(), buf_.data(), n_ * sizeof(T));
    buf_ = std::move(nb);
  }
  T& emplace_back() {
    if ((n_ + 1) * sizeof(T) > buf_.capacity()) reserve(std::max<size_t>(2 * n_, 1024));
    return *new (data() + n_++) T();
  }

 private:
  HugeBuf buf_;
  size_t n_ = 0;
};

// Bump allocator over a list of HugeBuf chunks; everything is freed together.
class HugeSlab {
 public:
  explicit HugeSlab(size_t chunk = size_t(16) << 20) : chunk_(chunk) {}
  // n bytes aligned to `align` (a power of two <= 64)
  uint8_t* alloc(size_t n, size_t align = 8) {
    size_t at = (used_ + align - 1) & ~(align - 1);
    if (chunks_.empty() || at + n > chunks_.back().capacity()) {
      chunks_.emplace_back(std::max(chunk_, n));
      at = 0;
    }
    used_ = at + n;
    return chunks_.back().data() + at;
  }
  void clear() {
    chunks_.clear();
    used_ = 0;
  }

 private:
  size_t chunk_;
  std::vector<HugeBuf> chunks_;
  size_t used_ = 0;
};

}  // namespace fcsg
