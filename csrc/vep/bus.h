// Frame bus: the node's cross-process frame store in shared memory, so any number of serving
// processes read any camera's frames with no hop through the process that decodes them.
//
// Reference parity: replaces the Redis stream every camera container XADDs its serialized
// VideoFrame into and the Go gRPC handler XREADs from (python/read_image.py:121,
// server/grpcapi/grpc_api.go:186-231). There, every decoded frame was serialized
// and pushed through Redis whether or not anyone read it; here frames stay in the owner's HBM
// ring (FrameRing) and are serialized into the bus only on demand:
//
//  * Owner (the process that decodes a camera: one per GPU, or per camera group): a control
//    segment /dev/shm/vep-bus.<tag>.<owner>.<pid> with one entry per camera (name, demand words
//    written by servers, supply words written by the owner) and, per camera, a data segment of
//    kSlots serialized-VideoFrame slots (page-locked, so the ring slot reaches it by one DMA).
//    A pump thread answers demand: when a camera has waiting readers and its ring holds a frame
//    newer than the bus's, it DMAs the ring slot behind the hand-encoded VideoFrame header into the
//    next bus slot, seqlock-commits it and wakes the readers (futex on the shared word).
//    The worker's publish hook keeps ring_seq current and rings the pump when readers wait.
//  * Reader (a serving process; no GPU context): maps every owner's control segment of the tag,
//    finds a camera by name, writes its demand (last_query / keyframe-only: the reference's
//    HSET last_access_time_<dev> / SET is_key_frame_only_<dev>, grpc_api.go:159-175), and copies
//    the newest bus slot out (one copy, into the bytes object grpcio sends), or takes a *lease*
//    on it (the native endpoint, rpcsrv.h): the owner does not rewrite a leased slot, so the
//    server writev()s the frame straight from shared memory with no copy at all. Every client of
//    a camera, in every serving process, shares the one DMA of a frame.
//
// Futexes on MAP_SHARED memory wake across processes; all shared words are lock-free atomics.
#pragma once

#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace vep {

class Worker;
class Camera;

namespace bus {

constexpr u64 kMagic = 0x32737562706576ull;  // "vepbus2"
constexpr int kNameLen = 96;
constexpr int kSlots = 4;  // newest + slots readers may still hold leases on + the one being written
// A lease pins a slot for at most this long (a reader that died holding one frees it then); the
// native endpoint closes a connection whose leased bytes are still unsent after kLeaseSendMs.
constexpr i64 kLeaseMs = 30000, kLeaseSendMs = 20000;

struct alignas(64) SlotHdr {
  std::atomic<u64> version;  // odd while the owner writes the slot
  std::atomic<i64> seq;      // ring sequence of the frame in it
  std::atomic<u64> len;      // serialized VideoFrame bytes
  // Readers sending straight from the slot (Reader::lease). The owner marks a slot odd, then
  // checks `leases` (seq_cst); a reader increments `leases`, then checks `version` (seq_cst): one
  // of the two always sees the other, so a leased slot is never rewritten.
  std::atomic<u32> leases;
  std::atomic<i64> lease_until;  // monotonic ms after which the leases are stale (dead reader)
};

struct alignas(64) CamEntry {
  std::atomic<u32> live;       // 1 while the camera is registered
  std::atomic<u32> gen;        // bumped on every (re)registration
  char name[kNameLen];
  // demand: written by readers
  std::atomic<i64> last_query_ms;
  std::atomic<u32> keyframe_only;  // 0 / 1; kUnset until a reader sets it
  std::atomic<u32> waiters;        // readers blocked on `pub`
  // supply: written by the owner
  std::atomic<u32> pub;            // futex word: +1 per bus publish or state change
  std::atomic<i64> ring_seq;       // newest sequence in the owner's HBM ring
  std::atomic<i64> bus_seq;        // sequence of the newest bus slot (0: none)
  std::atomic<u32> newest;         // slot holding bus_seq
  std::atomic<u32> data_gen;       // data segment generation (0: none yet)
  std::atomic<u64> slot_cap;       // bytes per slot of the data segment
  std::atomic<u32> pinned;         // the data segment is page-locked (the DMA lands in it directly)
  SlotHdr slots[kSlots];
};
constexpr u32 kUnset = 2;

struct alignas(64) Header {
  u64 magic;
  u32 max_cams;
  i32 owner_pid;
  std::atomic<u32> doorbell;       // futex: readers ring the owner's pump
  std::atomic<u64> heartbeat_ms;   // the pump's last pass (wall clock)
  std::atomic<u64> published;      // bus publishes (stats)
  char tag[64];
  CamEntry cams[1];                // [max_cams]
};

size_t control_bytes(int max_cams);
std::string shm_dir();

// ----------------------------------------------------------------------------- owner side
class Owner {
 public:
  // Creates the control segment vep-bus.<tag>.<owner>.<pid> for up to max_cams cameras.
  Owner(const std::string& tag, int owner, int max_cams);
  ~Owner();
  Owner(const Owner&) = delete;
  Owner& operator=(const Owner&) = delete;
  // Serve `w`'s cameras (installs the worker's publish hook, starts the pump thread).
  void attach(Worker* w);
  void add(int cam, const std::string& name);
  void remove(int cam);
  void stop();
  const std::string& path() const { return path_; }
  u64 published() const { return hdr_->published.load(); }
  u64 dma_bytes() const { return dma_bytes_.load(); }
  u64 lease_skips() const { return lease_skips_.load(); }  // publishes deferred: every other slot leased

 private:
  // One camera's data segment. Reference-counted: the pump holds a reference while its DMA
  // writes into the segment, so a camera removed / re-added meanwhile (remove(), add()) only
  // unlinks the file; the mapping (and its page-locking) goes when the last holder drops it.
  struct Mapping {
    Worker* w = nullptr;
    u8* base = nullptr;
    size_t bytes = 0;
    bool pinned = false;
    ~Mapping();
  };
  struct Data {
    std::string path;
    std::shared_ptr<Mapping> map;
    u64 ino = 0;
    u8* base() const { return map ? map->base : nullptr; }
    bool pinned() const { return map && map->pinned; }
  };
  void pump();
  void on_publish(int cam, i64 seq);
  void release_data(int cam);
  bool ensure_data(int cam, size_t slot_cap);
  std::string tag_;
  int owner_;
  std::string path_;
  u64 ino_ = 0;
  Header* hdr_ = nullptr;
  size_t bytes_ = 0;
  Worker* w_ = nullptr;
  std::vector<Data> data_;
  std::vector<i64> synced_query_;
  std::vector<u32> synced_kf_;
  std::vector<std::string> names_;
  std::mutex mu_;  // names_ / data_ against add / remove
  std::thread th_;
  std::atomic<bool> stop_{false};
  std::atomic<u64> dma_bytes_{0}, lease_skips_{0};
};

// ---------------------------------------------------------------------------- reader side
class Reader {
 public:
  explicit Reader(const std::string& tag);
  ~Reader();
  Reader(const Reader&) = delete;
  Reader& operator=(const Reader&) = delete;

  struct Ticket {  // a camera's bus frame that satisfied wait()
    std::shared_ptr<void> seg;  // keeps the control segment mapped
    int cam = -1;
    u32 gen = 0;
    i64 after = 0;
    size_t cap = 0;  // upper bound of the frame's length (the data segment's slot size)
  };
  // true if a live owner of the tag has `name` registered (rescans when not cached)
  bool has(const std::string& name);
  // Marks the demand (last_query = now; keyframe-only unless key_frame_only < 0: the reference's
  // HSET last_access_time_<dev> / SET is_key_frame_only_<dev>, grpc_api.go:159-175), then waits
  // up to wait_ms for a bus frame with seq > after that is at least as new as the owner's ring
  // was at the call. False: unknown camera or timeout.
  // touch = false: read only (no demand marked; an internal reader, not a client request).
  // cancel: when set (e.g. the client reset its stream), the wait ends within ~100 ms.
  bool wait(const std::string& name, i64 after, int wait_ms, int key_frame_only, Ticket* t, bool touch = true,
            const std::atomic<bool>* cancel = nullptr);
  // Copies the newest bus frame with seq > t.after into dst (cap >= t.cap): one seqlock-checked
  // memcpy. Returns its length and sequence, 0 if the camera went away meanwhile.
  size_t copy(const Ticket& t, u8* dst, size_t cap, i64* seq);
  // Sequence of the newest bus frame of the ticket's camera (a caller that already holds that
  // frame's bytes skips the copy).
  i64 newest_seq(const Ticket& t) const;
  // A lease on the newest bus frame with seq > t.after: its bytes in shared memory, not
  // rewritten while the lease lives (up to kLeaseMs), so a server sends them with no copy.
  // Null when there is none (or the camera went away). The lease keeps the segments mapped.
  struct Lease {
    const u8* data = nullptr;
    size_t len = 0;
    i64 seq = 0;
    i64 taken_ms = 0;  // monotonic ms
  };
  std::shared_ptr<const Lease> lease(const Ticket& t);
  u64 leases_taken() const { return leases_taken_.load(); }
  // Demand only.
  bool touch(const std::string& name, int key_frame_only);
  struct Info {
    int owner_pid = 0;
    bool pinned = false;
    i64 ring_seq = 0, bus_seq = 0;
    u64 published = 0;  // the owner's bus publishes (all its cameras)
  };
  bool info(const std::string& name, Info* out);
  std::vector<std::string> names();
  u64 rescans() const { return rescans_.load(); }
  // data segments this reader keeps mapped (tests: none outlives its camera or owner)
  size_t mapped_data_segments();

 private:
  struct Seg;
  struct Loc {
    std::shared_ptr<Seg> seg;
    int cam = -1;
    u32 gen = 0;
  };
  bool locate(const std::string& name, Loc* loc);
  void rescan_locked();
  std::string tag_;
  std::mutex mu_;
  std::vector<std::shared_ptr<Seg>> segs_;
  std::unordered_map<std::string, Loc> where_;
  // Mapped data segments, key: control segment path + '/' + cam. An entry is unmapped when its
  // camera is re-registered or removed (gen / live), or its owner's control segment disappears:
  // an unlinked tmpfs file keeps its pages while any process maps it.
  struct DataMap {
    std::string seg_path;
    int cam = -1;
    u32 data_gen = 0, cam_gen = 0;
    std::shared_ptr<void> map;
  };
  std::unordered_map<std::string, DataMap> data_;
  void prune_data_locked();
  i64 last_scan_ms_ = 0;
  std::atomic<u64> rescans_{0}, leases_taken_{0};
  std::shared_ptr<void> data_map(const std::shared_ptr<Seg>& seg, int cam, u32 gen, u32 dg, u64 scap);
};

// Removes the bus segments a (dead) process left in /dev/shm. Returns how many.
int remove_segments_of(int pid);

}  // namespace bus
}  // namespace vep
