// Single-producer / multi-consumer ring of fixed-size int64 records in POSIX shared memory
// (SURVEY §5 "use shared-memory rings rather than sockets" for the control hop between the
// processes of one node).
//
// Used for the tensor-parallel step header: the TP driver publishes one record per engine
// step (op, tokens, sequences, bucket, ...) and every follower rank of the group reads it
// before replaying the same hipGraph. Replaces a gloo broadcast over TCP (tens of
// microseconds per step) with a store + a release-ordered sequence
// number that the followers poll (sub-microsecond when they are already waiting).
//
// Layout of the segment: a control block (magic, geometry, the published sequence number),
// one cache line per consumer for its acknowledged sequence number (the producer never
// overwrites a slot a consumer has not read), then `slots` records of `ints` int64 each.
#pragma once
#include <atomic>
#include <cstdint>
#include <string>

namespace rt {

class ShmRing {
 public:
  // create = true: the producer creates (and finally unlinks) the segment; consumers attach,
  // retrying for up to `attach_timeout_s` while the producer has not created it yet.
  ShmRing(const std::string& name, int ints, int slots, int consumers, bool create,
          double attach_timeout_s = 60.0);
  ~ShmRing();
  ShmRing(const ShmRing&) = delete;
  ShmRing& operator=(const ShmRing&) = delete;

  // producer: append one record (blocks while the slowest consumer is `slots` records
  // behind; returns false after timeout_s)
  bool put(const int64_t* rec, double timeout_s = 600.0);
  // consumer `c`: copy the next record into rec (blocks up to timeout_s; false on timeout)
  bool get(int c, int64_t* rec, double timeout_s = 600.0);
  int64_t published() const;
  int ints() const { return ints_; }
  void unlink();

 private:
  struct Ctl {
    uint64_t magic;
    int32_t ints, slots, consumers, pad;
    alignas(64) std::atomic<int64_t> seq;  // records published
  };
  struct alignas(64) Ack {
    std::atomic<int64_t> seq;  // records consumed by this consumer
  };
  std::string name_;
  int ints_, slots_, consumers_;
  bool owner_;
  size_t bytes_ = 0;
  void* base_ = nullptr;
  Ctl* ctl_ = nullptr;
  Ack* acks_ = nullptr;
  int64_t* recs_ = nullptr;
  int64_t next_ = 0;  // producer: next sequence number; consumer reads track acks_[c]
};

// All-gather of byte payloads between the `world` processes of one node through POSIX shared
// memory: the host control plane of the node-wide semantic store (pilottai_amd/memory/
// node_store.py), whose per-round headers, filters and items are tiny and latency-bound (a gloo
// all-gather over loopback TCP costs milliseconds at 8 ranks; this costs microseconds).
//
// Layout: a control block, one cache line per rank (arrive / done round counters and the
// payload sizes of the two banks), then two banks of `world` slots of `slot_bytes` each. Round
// s (1-based) uses bank s & 1; a rank writes its slot only once every rank has finished reading
// round s - 2 (the bank's previous use), publishes it with a release store of arrive = s, waits
// for arrive >= s on every rank (acquire), copies all slots out and marks done = s.
class ShmGather {
 public:
  ShmGather(const std::string& name, int world, int rank, size_t slot_bytes, bool create,
            double attach_timeout_s = 60.0);
  ~ShmGather();
  ShmGather(const ShmGather&) = delete;
  ShmGather& operator=(const ShmGather&) = delete;

  // in: n <= slot_bytes bytes; out: world * slot_bytes bytes (rank q's payload at q * slot_bytes);
  // sizes: world entries. Returns false on timeout (a peer died or left).
  bool all_gather(const void* in, size_t n, void* out, int64_t* sizes, double timeout_s);
  // The same round in two halves, for callers that read the payloads in place: publish() writes
  // this rank's slot and waits for every rank's; then peer(q) / peer_size(q) point into the
  // segment until finish() releases the bank.
  bool publish(const void* in, size_t n, double timeout_s);
  const char* peer(int q) const;
  int64_t peer_size(int q) const;
  void finish();
  double waited_s() const { return waited_; }  // total time spent waiting for peers
  size_t slot_bytes() const { return slot_; }
  int world() const { return world_; }
  int rank() const { return rank_; }
  void unlink();

 private:
  struct Ctl {
    uint64_t magic;
    int64_t world, slot;
  };
  struct alignas(64) Peer {
    std::atomic<int64_t> arrive;
    std::atomic<int64_t> done;
    int64_t size[2];
  };
  std::string name_;
  int world_, rank_;
  size_t slot_;
  bool owner_;
  size_t bytes_ = 0;
  void* base_ = nullptr;
  Ctl* ctl_ = nullptr;
  Peer* peers_ = nullptr;
  char* data_ = nullptr;
  int64_t round_ = 0;
  double waited_ = 0.0;
};

}  // namespace rt
