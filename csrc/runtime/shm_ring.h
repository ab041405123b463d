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

}  // namespace rt
