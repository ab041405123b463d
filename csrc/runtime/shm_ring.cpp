// POSIX shared-memory header ring (see shm_ring.h).
#include "shm_ring.h"

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace rt {

namespace {
constexpr uint64_t kMagic = 0x70696c6f74726e67ULL;  // "pilotrng"

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// spin briefly, then yield, then sleep in growing steps: a waiting follower answers within
// microseconds while the driver is busy, and burns little CPU while the engine is idle
struct Backoff {
  int n = 0;
  void wait() {
    ++n;
    if (n < 2000) {
#if defined(__x86_64__)
      __builtin_ia32_pause();
#endif
    } else if (n < 4000) {
      sched_yield();
    } else {
      std::this_thread::sleep_for(std::chrono::microseconds(n < 8000 ? 20 : 200));
    }
  }
};

size_t round_up(size_t v, size_t a) { return (v + a - 1) / a * a; }
}  // namespace

ShmRing::ShmRing(const std::string& name, int ints, int slots, int consumers, bool create,
                 double attach_timeout_s)
    : name_(name.empty() || name[0] == '/' ? name : "/" + name), ints_(ints), slots_(slots),
      consumers_(consumers), owner_(create) {
  if (ints <= 0 || slots <= 0 || consumers <= 0) throw std::invalid_argument("ShmRing geometry must be positive");
  const size_t ctl = round_up(sizeof(Ctl), 64);
  const size_t acks = sizeof(Ack) * (size_t)consumers;
  bytes_ = ctl + acks + sizeof(int64_t) * (size_t)ints * (size_t)slots;
  int fd = -1;
  if (create) {
    shm_unlink(name_.c_str());  // a stale segment of a crashed run
    fd = shm_open(name_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("shm_open(create) failed for " + name_);
    if (ftruncate(fd, (off_t)bytes_) != 0) {
      close(fd);
      shm_unlink(name_.c_str());
      throw std::runtime_error("ftruncate failed for " + name_);
    }
  } else {
    const double t0 = now_s();
    Backoff b;
    while (true) {
      fd = shm_open(name_.c_str(), O_RDWR, 0600);
      if (fd >= 0) {
        struct stat st;
        if (fstat(fd, &st) == 0 && (size_t)st.st_size >= bytes_) break;
        close(fd);
        fd = -1;
      }
      if (now_s() - t0 > attach_timeout_s) throw std::runtime_error("timed out attaching to " + name_);
      b.wait();
    }
  }
  base_ = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (base_ == MAP_FAILED) {
    base_ = nullptr;
    throw std::runtime_error("mmap failed for " + name_);
  }
  ctl_ = reinterpret_cast<Ctl*>(base_);
  acks_ = reinterpret_cast<Ack*>(static_cast<char*>(base_) + ctl);
  recs_ = reinterpret_cast<int64_t*>(static_cast<char*>(base_) + ctl + acks);
  if (create) {
    std::memset(base_, 0, bytes_);
    ctl_->ints = ints;
    ctl_->slots = slots;
    ctl_->consumers = consumers;
    for (int c = 0; c < consumers; ++c) acks_[c].seq.store(0, std::memory_order_relaxed);
    ctl_->seq.store(0, std::memory_order_relaxed);
    std::atomic_thread_fence(std::memory_order_release);
    reinterpret_cast<std::atomic<uint64_t>*>(&ctl_->magic)->store(kMagic, std::memory_order_release);
  } else {
    const double t0 = now_s();
    Backoff b;
    while (reinterpret_cast<std::atomic<uint64_t>*>(&ctl_->magic)->load(std::memory_order_acquire) != kMagic) {
      if (now_s() - t0 > attach_timeout_s) throw std::runtime_error("ring " + name_ + " never initialised");
      b.wait();
    }
    if (ctl_->ints != ints || ctl_->slots != slots || ctl_->consumers != consumers)
      throw std::runtime_error("ring " + name_ + " geometry mismatch");
  }
}

ShmRing::~ShmRing() {
  if (base_) munmap(base_, bytes_);
  if (owner_) shm_unlink(name_.c_str());
}

void ShmRing::unlink() { shm_unlink(name_.c_str()); }

int64_t ShmRing::published() const { return ctl_->seq.load(std::memory_order_acquire); }

bool ShmRing::put(const int64_t* rec, double timeout_s) {
  const int64_t s = next_;
  const double t0 = now_s();
  Backoff b;
  for (int c = 0; c < consumers_; ++c)  // never overwrite a record a consumer has not read
    while (acks_[c].seq.load(std::memory_order_acquire) <= s - slots_) {
      if (now_s() - t0 > timeout_s) return false;
      b.wait();
    }
  std::memcpy(recs_ + (size_t)(s % slots_) * ints_, rec, sizeof(int64_t) * ints_);
  ctl_->seq.store(s + 1, std::memory_order_release);  // publishes the record
  next_ = s + 1;
  return true;
}

bool ShmRing::get(int c, int64_t* rec, double timeout_s) {
  if (c < 0 || c >= consumers_) throw std::out_of_range("consumer index");
  const int64_t s = acks_[c].seq.load(std::memory_order_relaxed);
  const double t0 = now_s();
  Backoff b;
  while (ctl_->seq.load(std::memory_order_acquire) <= s) {
    if (now_s() - t0 > timeout_s) return false;
    b.wait();
  }
  std::memcpy(rec, recs_ + (size_t)(s % slots_) * ints_, sizeof(int64_t) * ints_);
  acks_[c].seq.store(s + 1, std::memory_order_release);  // the slot may be reused
  return true;
}

}  // namespace rt
