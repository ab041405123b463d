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

namespace {
constexpr uint64_t kGatherMagic = 0x70696c6f74676174ULL;  // "pilotgat"

void* map_segment(const std::string& name, size_t bytes, bool create, double attach_timeout_s) {
  int fd = -1;
  if (create) {
    shm_unlink(name.c_str());
    fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("shm_open(create) failed for " + name);
    if (ftruncate(fd, (off_t)bytes) != 0) {
      close(fd);
      shm_unlink(name.c_str());
      throw std::runtime_error("ftruncate failed for " + name);
    }
  } else {
    const double t0 = now_s();
    Backoff b;
    while (true) {
      fd = shm_open(name.c_str(), O_RDWR, 0600);
      if (fd >= 0) {
        struct stat st;
        if (fstat(fd, &st) == 0 && (size_t)st.st_size >= bytes) break;
        close(fd);
        fd = -1;
      }
      if (now_s() - t0 > attach_timeout_s) throw std::runtime_error("timed out attaching to " + name);
      b.wait();
    }
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) throw std::runtime_error("mmap failed for " + name);
  return p;
}
}  // namespace

ShmGather::ShmGather(const std::string& name, int world, int rank, size_t slot_bytes, bool create,
                     double attach_timeout_s)
    : name_(name.empty() || name[0] == '/' ? name : "/" + name), world_(world), rank_(rank),
      slot_(round_up(slot_bytes, 64)), owner_(create) {
  if (world <= 0 || rank < 0 || rank >= world || slot_bytes == 0)
    throw std::invalid_argument("ShmGather geometry");
  const size_t ctl = round_up(sizeof(Ctl), 64);
  const size_t peers = sizeof(Peer) * (size_t)world;
  bytes_ = ctl + peers + 2 * (size_t)world * slot_;
  base_ = map_segment(name_, bytes_, create, attach_timeout_s);
  ctl_ = reinterpret_cast<Ctl*>(base_);
  peers_ = reinterpret_cast<Peer*>(static_cast<char*>(base_) + ctl);
  data_ = static_cast<char*>(base_) + ctl + peers;
  auto* magic = reinterpret_cast<std::atomic<uint64_t>*>(&ctl_->magic);
  if (create) {
    std::memset(base_, 0, ctl + peers);  // the data banks are zero pages already
    ctl_->world = world;
    ctl_->slot = (int64_t)slot_;
    for (int q = 0; q < world; ++q) {
      peers_[q].arrive.store(0, std::memory_order_relaxed);
      peers_[q].done.store(0, std::memory_order_relaxed);
    }
    std::atomic_thread_fence(std::memory_order_release);
    magic->store(kGatherMagic, std::memory_order_release);
  } else {
    const double t0 = now_s();
    Backoff b;
    while (magic->load(std::memory_order_acquire) != kGatherMagic) {
      if (now_s() - t0 > attach_timeout_s) throw std::runtime_error("gather " + name_ + " never initialised");
      b.wait();
    }
    if (ctl_->world != world || ctl_->slot != (int64_t)slot_)
      throw std::runtime_error("gather " + name_ + " geometry mismatch");
  }
}

ShmGather::~ShmGather() {
  if (base_) munmap(base_, bytes_);
  if (owner_) shm_unlink(name_.c_str());
}

void ShmGather::unlink() { shm_unlink(name_.c_str()); }

bool ShmGather::publish(const void* in, size_t n, double timeout_s) {
  if (n > slot_) throw std::length_error("ShmGather payload larger than the slot");
  const int64_t s = round_ + 1;
  const int bank = (int)(s & 1);
  const double t0 = now_s();
  Backoff b;
  // the bank's previous use (round s - 2) must be fully read by every rank
  for (int q = 0; q < world_; ++q)
    while (peers_[q].done.load(std::memory_order_acquire) < s - 2) {
      if (now_s() - t0 > timeout_s) return false;
      b.wait();
    }
  const double t1 = now_s();
  char* mine = data_ + ((size_t)bank * world_ + rank_) * slot_;
  if (n) std::memcpy(mine, in, n);
  peers_[rank_].size[bank] = (int64_t)n;
  peers_[rank_].arrive.store(s, std::memory_order_release);
  const double t2 = now_s();
  for (int q = 0; q < world_; ++q)
    while (peers_[q].arrive.load(std::memory_order_acquire) < s) {
      if (now_s() - t0 > timeout_s) return false;
      b.wait();
    }
  waited_ += (t1 - t0) + (now_s() - t2);
  round_ = s;
  return true;
}

const char* ShmGather::peer(int q) const {
  return data_ + ((size_t)(round_ & 1) * world_ + q) * slot_;
}

int64_t ShmGather::peer_size(int q) const { return peers_[q].size[round_ & 1]; }

void ShmGather::finish() { peers_[rank_].done.store(round_, std::memory_order_release); }

bool ShmGather::all_gather(const void* in, size_t n, void* out, int64_t* sizes, double timeout_s) {
  if (!publish(in, n, timeout_s)) return false;
  char* o = static_cast<char*>(out);
  for (int q = 0; q < world_; ++q) {
    sizes[q] = peer_size(q);
    if (sizes[q]) std::memcpy(o + (size_t)q * slot_, peer(q), (size_t)sizes[q]);
  }
  finish();
  return true;
}

}  // namespace rt
