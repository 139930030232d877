// Frame bus: see bus.h.
#include "bus.h"

#include <dirent.h>
#include <fcntl.h>
#include <linux/futex.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <climits>
#include <cstring>
#include <ctime>

#include "runtime.h"

namespace vep::bus {

static_assert(std::atomic<u64>::is_always_lock_free && std::atomic<u32>::is_always_lock_free,
              "bus words must be lock-free to be shared between processes");

namespace {

i64 wall_ms() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return i64(ts.tv_sec) * 1000 + ts.tv_nsec / 1000000;
}

i64 mono_ms() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return i64(ts.tv_sec) * 1000 + ts.tv_nsec / 1000000;
}

// Shared (not FUTEX_PRIVATE) futex ops: the words live in MAP_SHARED segments of several processes.
void futex_wait(std::atomic<u32>* w, u32 expect, int timeout_ms) {
  timespec ts{timeout_ms / 1000, long(timeout_ms % 1000) * 1000000L};
  syscall(SYS_futex, reinterpret_cast<u32*>(w), FUTEX_WAIT, expect, &ts, nullptr, 0);
}

void futex_wake(std::atomic<u32>* w) { syscall(SYS_futex, reinterpret_cast<u32*>(w), FUTEX_WAKE, INT_MAX, nullptr, nullptr, 0); }

std::string clean_tag(const std::string& t) {
  std::string s;
  for (char c : t) s.push_back(std::isalnum(static_cast<unsigned char>(c)) || c == '-' || c == '_' ? c : '_');
  VEP_CHECK(!s.empty() && s.size() < 48, "bus tag must be 1..47 characters");
  return s;
}

void* map_file(const std::string& path, size_t bytes, bool create, bool writable) {
  const int fd = ::open(path.c_str(), create ? (O_RDWR | O_CREAT | O_EXCL) : (writable ? O_RDWR : O_RDONLY), 0600);
  if (fd < 0) return nullptr;
  if (create && ::ftruncate(fd, off_t(bytes)) != 0) {
    ::close(fd);
    ::unlink(path.c_str());
    return nullptr;
  }
  void* p = ::mmap(nullptr, bytes, writable ? (PROT_READ | PROT_WRITE) : PROT_READ, MAP_SHARED, fd, 0);
  ::close(fd);
  return p == MAP_FAILED ? nullptr : p;
}

bool pid_alive(int pid) { return pid > 0 && (::kill(pid, 0) == 0 || errno == EPERM); }

u64 inode_of(const std::string& path) {
  struct stat st;
  return ::stat(path.c_str(), &st) == 0 ? u64(st.st_ino) : 0;
}

// unlink `path` only if it is still the file this process created (inode `ino`): another owner
// with the same name may have replaced it since
void unlink_own(const std::string& path, u64 ino) {
  if (ino && inode_of(path) == ino) ::unlink(path.c_str());
}

}  // namespace

size_t control_bytes(int max_cams) {
  return sizeof(Header) + sizeof(CamEntry) * size_t(std::max(0, max_cams - 1));
}

std::string shm_dir() {
  struct stat st;
  return ::stat("/dev/shm", &st) == 0 && S_ISDIR(st.st_mode) ? "/dev/shm" : "/tmp";
}

int remove_segments_of(int pid) {
  const std::string dir = shm_dir(), mark = "." + std::to_string(pid);
  int n = 0;
  DIR* d = ::opendir(dir.c_str());
  if (!d) return 0;
  while (dirent* e = ::readdir(d)) {
    const std::string f = e->d_name;
    if (f.rfind("vep-bus.", 0) != 0) continue;
    // vep-bus.<tag>.<owner>.<pid>[.c<cam>.g<gen>]
    std::vector<std::string> parts;
    size_t a = 0;
    for (size_t b; (b = f.find('.', a)) != std::string::npos; a = b + 1) parts.push_back(f.substr(a, b - a));
    parts.push_back(f.substr(a));
    if (parts.size() >= 4 && parts[3] == std::to_string(pid) && ::unlink((dir + "/" + f).c_str()) == 0) ++n;
  }
  ::closedir(d);
  return n;
}

// ------------------------------------------------------------------------------------ Owner

Owner::Owner(const std::string& tag, int owner, int max_cams) : tag_(clean_tag(tag)), owner_(owner) {
  VEP_CHECK(max_cams >= 1 && max_cams <= 4096, "bus: max_cams out of range");
  path_ = shm_dir() + "/vep-bus." + tag_ + "." + std::to_string(owner) + "." + std::to_string(::getpid());
  ::unlink(path_.c_str());  // (a previous owner of this pid cannot be alive)
  bytes_ = control_bytes(max_cams);
  // the header and entries are built in a private staging copy, then published by rename: a
  // reader never maps a half-initialised segment
  const std::string tmp = path_ + ".tmp";
  ::unlink(tmp.c_str());
  void* p = map_file(tmp, bytes_, true, true);
  VEP_CHECK(p, "bus: cannot create " + tmp + ": " + std::strerror(errno));
  hdr_ = static_cast<Header*>(p);  // zero-filled by ftruncate
  hdr_->max_cams = u32(max_cams);
  hdr_->owner_pid = ::getpid();
  std::snprintf(hdr_->tag, sizeof(hdr_->tag), "%s", tag_.c_str());
  for (int i = 0; i < max_cams; ++i) hdr_->cams[i].keyframe_only.store(kUnset);
  std::atomic_thread_fence(std::memory_order_release);
  hdr_->magic = kMagic;
  VEP_CHECK(::rename(tmp.c_str(), path_.c_str()) == 0, "bus: cannot publish " + path_);
  ino_ = inode_of(path_);
  data_.resize(size_t(max_cams));
  synced_query_.assign(size_t(max_cams), 0);
  synced_kf_.assign(size_t(max_cams), kUnset);
  names_.resize(size_t(max_cams));
}

Owner::~Owner() {
  stop();
  for (size_t i = 0; i < data_.size(); ++i) release_data(int(i));
  if (hdr_) {
    ::munmap(hdr_, bytes_);
    unlink_own(path_, ino_);
  }
}

void Owner::attach(Worker* w) {
  VEP_CHECK(!w_, "bus owner already attached");
  w_ = w;
  w_->set_publish_hook([this](int cam, i64 seq) { on_publish(cam, seq); });
  th_ = std::thread([this] {
    name_thread("vep-pump");
    pin_current_thread(w_->host_domain().cpus);  // (the worker's host domain)
    pump();
  });
}

void Owner::stop() {
  if (stop_.exchange(true)) return;
  if (w_) w_->set_publish_hook(nullptr);
  hdr_->doorbell.fetch_add(1);
  futex_wake(&hdr_->doorbell);
  if (th_.joinable()) th_.join();
  for (u32 i = 0; i < hdr_->max_cams; ++i) {  // waiting readers give up at once
    hdr_->cams[i].live.store(0);
    hdr_->cams[i].pub.fetch_add(1);
    futex_wake(&hdr_->cams[i].pub);
  }
}

void Owner::add(int cam, const std::string& name) {
  VEP_CHECK(cam >= 0 && u32(cam) < hdr_->max_cams, "bus: camera index out of range");
  VEP_CHECK(name.size() < size_t(kNameLen), "bus: camera name too long");
  std::lock_guard<std::mutex> g(mu_);
  release_data(cam);
  CamEntry& e = hdr_->cams[cam];
  e.live.store(0, std::memory_order_release);
  std::memset(e.name, 0, sizeof(e.name));
  std::memcpy(e.name, name.data(), name.size());
  e.last_query_ms.store(0);
  e.keyframe_only.store(kUnset);
  e.waiters.store(0);
  e.ring_seq.store(0);
  e.bus_seq.store(0);
  e.newest.store(0);
  // (data_gen stays monotonic per entry: a reader's cached mapping of an older camera's segment
  // never matches the generation of this one's)
  for (auto& s : e.slots) {
    s.version.store(0);
    s.seq.store(0);
    s.len.store(0);
  }
  synced_query_[size_t(cam)] = 0;
  synced_kf_[size_t(cam)] = kUnset;
  names_[size_t(cam)] = name;
  e.gen.fetch_add(1, std::memory_order_acq_rel);
  e.live.store(1, std::memory_order_release);
}

void Owner::remove(int cam) {
  if (cam < 0 || u32(cam) >= hdr_->max_cams) return;
  std::lock_guard<std::mutex> g(mu_);
  CamEntry& e = hdr_->cams[cam];
  e.live.store(0, std::memory_order_release);
  e.gen.fetch_add(1, std::memory_order_acq_rel);
  names_[size_t(cam)].clear();
  e.pub.fetch_add(1);
  futex_wake(&e.pub);
  release_data(cam);
}

Owner::Mapping::~Mapping() {
  if (!base) return;
  if (pinned && w) w->unregister_host(base);
  ::munmap(base, bytes);
}

void Owner::release_data(int cam) {
  Data& d = data_[size_t(cam)];
  if (!d.map) return;
  unlink_own(d.path, d.ino);  // readers that still map it keep their mapping
  d = Data{};                 // (the pump's in-flight DMA may still hold the mapping)
}

bool Owner::ensure_data(int cam, size_t slot_cap) {
  CamEntry& e = hdr_->cams[cam];
  Data& d = data_[size_t(cam)];
  if (d.map && e.slot_cap.load() >= slot_cap) return true;
  release_data(cam);
  const u32 gen = e.data_gen.load() + 1;
  const size_t cap = (slot_cap + 4095) & ~size_t(4095);
  Data nd;
  nd.path = path_ + ".c" + std::to_string(cam) + ".g" + std::to_string(gen);
  auto m = std::make_shared<Mapping>();
  m->bytes = cap * kSlots;
  ::unlink(nd.path.c_str());
  void* p = map_file(nd.path, m->bytes, true, true);
  if (!p) return false;
  m->base = static_cast<u8*>(p);
  m->w = w_;
  nd.ino = inode_of(nd.path);
  m->pinned = w_ && w_->register_host(m->base, m->bytes);
  nd.map = std::move(m);
  d = nd;
  for (auto& s : e.slots) {
    s.version.fetch_add(2);  // (even: no reader may trust an old slot of the previous segment)
    s.seq.store(0);
    s.len.store(0);
  }
  e.bus_seq.store(0);
  e.slot_cap.store(cap);
  e.pinned.store(nd.pinned() ? 1u : 0u);
  e.data_gen.store(gen, std::memory_order_release);
  return true;
}

void Owner::on_publish(int cam, i64 seq) {
  if (cam < 0 || u32(cam) >= hdr_->max_cams) return;
  CamEntry& e = hdr_->cams[cam];
  e.ring_seq.store(seq, std::memory_order_release);
  if (e.waiters.load(std::memory_order_acquire) > 0) {
    hdr_->doorbell.fetch_add(1, std::memory_order_acq_rel);
    futex_wake(&hdr_->doorbell);
  }
}

void Owner::pump() {
  if (w_->device().gpu()) w_->device().bind();
  struct Job {
    int cam, slot;
    size_t pre;
    std::string name;
    std::shared_ptr<FrameRing> ring;
    std::shared_ptr<Camera> keep;
    std::shared_ptr<Mapping> map;  // the segment the DMA writes into (kept mapped until it is done)
  };
  std::vector<Job> jobs;
  std::vector<Worker::ReadReq> reqs;
  while (!stop_.load()) {
    const u32 db = hdr_->doorbell.load(std::memory_order_acquire);
    hdr_->heartbeat_ms.store(u64(wall_ms()));
    jobs.clear();
    reqs.clear();
    {
      std::lock_guard<std::mutex> g(mu_);
      for (u32 i = 0; i < hdr_->max_cams; ++i) {
        if (names_[i].empty()) continue;
        CamEntry& e = hdr_->cams[i];
        std::shared_ptr<Camera> c = w_->camera(int(i));
        if (!c) continue;
        // demand -> the camera's control atomics (the lazy decoder reads them per packet)
        const i64 lq = e.last_query_ms.load(std::memory_order_acquire);
        if (lq > synced_query_[i]) {
          synced_query_[i] = lq;
          if (lq > c->last_query_ms.load()) c->last_query_ms.store(lq);
        }
        const u32 kf = e.keyframe_only.load(std::memory_order_acquire);
        if (kf != kUnset && kf != synced_kf_[i]) {
          synced_kf_[i] = kf;
          c->keyframe_only.store(kf == 1);
        }
        std::shared_ptr<FrameRing> ring = c->ring();
        if (!ring) continue;
        const i64 rs = ring->published();
        e.ring_seq.store(rs, std::memory_order_release);
        if (e.waiters.load(std::memory_order_acquire) == 0 || rs <= e.bus_seq.load(std::memory_order_acquire)) continue;
        const size_t n = ring->slot_bytes();
        FrameMeta probe{};
        probe.width = ring->width();
        probe.height = ring->height();
        const std::string pre = encode_video_frame(probe, n, names_[i]).first;
        if (!ensure_data(int(i), pre.size() + n + video_frame_suffix_max(names_[i]))) continue;
        const u64 cap = e.slot_cap.load();
        // the next slot after the newest that no reader holds a lease on (marked odd first,
        // then the leases checked: see SlotHdr)
        int slot = -1;
        const bool none = e.bus_seq.load() == 0;
        const int newest = int(e.newest.load() % kSlots);
        for (int d = none ? 0 : 1; d < kSlots && slot < 0; ++d) {
          const int k = (newest + d) % kSlots;
          SlotHdr& s = e.slots[k];
          s.version.fetch_add(1, std::memory_order_seq_cst);  // odd: being written
          if (s.leases.load(std::memory_order_seq_cst) > 0 && mono_ms() < s.lease_until.load(std::memory_order_acquire)) {
            s.version.fetch_add(1, std::memory_order_acq_rel);  // (even again: untouched)
            continue;
          }
          slot = k;
        }
        if (slot < 0) {  // every other slot is being sent by some reader: the next pass retries
          lease_skips_.fetch_add(1);
          continue;
        }
        u8* dst = data_[i].base() + size_t(slot) * cap;
        std::memcpy(dst, pre.data(), pre.size());
        jobs.push_back({int(i), slot, pre.size(), names_[i], ring, c, data_[i].map});
        Worker::ReadReq r;
        r.ring = ring.get();
        r.after = e.bus_seq.load();
        r.dst = dst + pre.size();
        r.cap = n;
        r.pinned = data_[i].pinned();
        reqs.push_back(r);
      }
    }
    if (jobs.empty()) {
      futex_wait(&hdr_->doorbell, db, 20);
      continue;
    }
    try {
      w_->read_latest_many(reqs);
    } catch (const std::exception&) {
      for (auto& r : reqs) r.ok = false;
    }
    std::lock_guard<std::mutex> g(mu_);
    for (size_t k = 0; k < jobs.size(); ++k) {
      const Job& j = jobs[k];
      CamEntry& e = hdr_->cams[j.cam];
      SlotHdr& s = e.slots[j.slot];
      // (the same segment as at the start: not replaced by a remove / add / regrow meanwhile)
      if (reqs[k].ok && names_[size_t(j.cam)] == j.name && data_[size_t(j.cam)].map == j.map) {
        const size_t n = j.ring->slot_bytes();
        const std::string suf = encode_video_frame(reqs[k].meta, n, j.name).second;
        u8* dst = j.map->base + size_t(j.slot) * e.slot_cap.load();
        std::memcpy(dst + j.pre + n, suf.data(), suf.size());
        s.len.store(j.pre + n + suf.size(), std::memory_order_relaxed);
        s.seq.store(reqs[k].meta.seq, std::memory_order_relaxed);
        s.version.fetch_add(1, std::memory_order_acq_rel);  // even: stable
        e.newest.store(u32(j.slot), std::memory_order_release);
        e.bus_seq.store(reqs[k].meta.seq, std::memory_order_release);
        hdr_->published.fetch_add(1);
        dma_bytes_.fetch_add(n);
      } else {
        s.seq.store(0);
        s.version.fetch_add(1, std::memory_order_acq_rel);
      }
      e.pub.fetch_add(1, std::memory_order_acq_rel);
      futex_wake(&e.pub);
    }
  }
}

// ----------------------------------------------------------------------------------- Reader

struct Reader::Seg {
  std::string path;
  Header* hdr = nullptr;
  size_t bytes = 0;
  int pid = 0;
  ~Seg() {
    if (hdr) ::munmap(hdr, bytes);
  }
};

namespace {
struct DataSeg {  // one mapped data segment (shared by the copies in flight)
  const u8* base = nullptr;
  size_t bytes = 0;
  ~DataSeg() {
    if (base) ::munmap(const_cast<u8*>(base), bytes);
  }
};
}  // namespace

Reader::Reader(const std::string& tag) : tag_(clean_tag(tag)) {}

Reader::~Reader() = default;

void Reader::rescan_locked() {
  rescans_.fetch_add(1);
  last_scan_ms_ = mono_ms();
  const std::string dir = shm_dir(), pre = "vep-bus." + tag_ + ".";
  std::vector<std::shared_ptr<Seg>> keep;
  DIR* d = ::opendir(dir.c_str());
  if (!d) return;
  while (dirent* ent = ::readdir(d)) {
    const std::string f = ent->d_name;
    if (f.rfind(pre, 0) != 0) continue;
    const std::string rest = f.substr(pre.size());  // <owner>.<pid>
    const size_t dot = rest.find('.');
    if (dot == std::string::npos || rest.find('.', dot + 1) != std::string::npos) continue;
    const int pid = std::atoi(rest.c_str() + dot + 1);
    if (!pid_alive(pid)) continue;
    const std::string path = dir + "/" + f;
    std::shared_ptr<Seg> have;
    for (auto& s : segs_)
      if (s->path == path && s->pid == pid) have = s;
    if (!have) {
      struct stat st;
      if (::stat(path.c_str(), &st) != 0 || size_t(st.st_size) < sizeof(Header)) continue;
      void* p = map_file(path, size_t(st.st_size), false, true);
      if (!p) continue;
      auto s = std::make_shared<Seg>();
      s->path = path;
      s->hdr = static_cast<Header*>(p);
      s->bytes = size_t(st.st_size);
      s->pid = pid;
      if (s->hdr->magic != kMagic || control_bytes(int(s->hdr->max_cams)) > s->bytes) continue;
      have = s;
    }
    keep.push_back(have);
  }
  ::closedir(d);
  segs_.swap(keep);
  where_.clear();
  prune_data_locked();
  for (auto& s : segs_)
    for (u32 i = 0; i < s->hdr->max_cams; ++i) {
      const CamEntry& e = s->hdr->cams[i];
      const u32 gen = e.gen.load(std::memory_order_acquire);
      if (!e.live.load(std::memory_order_acquire)) continue;
      std::string name(e.name, strnlen(e.name, sizeof(e.name)));
      if (e.gen.load(std::memory_order_acquire) != gen || name.empty()) continue;
      where_[name] = Loc{s, int(i), gen};
    }
}

void Reader::prune_data_locked() {
  for (auto it = data_.begin(); it != data_.end();) {
    const Seg* seg = nullptr;
    for (const auto& sp : segs_)
      if (sp->path == it->second.seg_path) seg = sp.get();
    bool keep = seg != nullptr && it->second.cam >= 0 && u32(it->second.cam) < seg->hdr->max_cams;
    if (keep) {
      const CamEntry& e = seg->hdr->cams[it->second.cam];
      keep = e.live.load(std::memory_order_acquire) && e.gen.load(std::memory_order_acquire) == it->second.cam_gen &&
             e.data_gen.load(std::memory_order_acquire) == it->second.data_gen;
    }
    it = keep ? std::next(it) : data_.erase(it);  // (a copy in flight holds its own reference)
  }
}

size_t Reader::mapped_data_segments() {
  std::lock_guard<std::mutex> g(mu_);
  rescan_locked();
  return data_.size();
}

bool Reader::locate(const std::string& name, Loc* loc) {
  std::lock_guard<std::mutex> g(mu_);
  // (a periodic rescan also unmaps the data segments of cameras and owners that went away)
  if (mono_ms() - last_scan_ms_ >= 5000) rescan_locked();
  for (int pass = 0; pass < 2; ++pass) {
    auto it = where_.find(name);
    if (it != where_.end()) {
      const Loc& l = it->second;
      const CamEntry& e = l.seg->hdr->cams[l.cam];
      if (e.live.load(std::memory_order_acquire) && e.gen.load(std::memory_order_acquire) == l.gen &&
          pid_alive(l.seg->pid)) {
        *loc = l;
        return true;
      }
    }
    // unknown or stale (camera moved, owner restarted): rescan, at most every 20 ms for misses
    if (pass == 0 && (it != where_.end() || mono_ms() - last_scan_ms_ >= 20)) rescan_locked();
    else break;
  }
  return false;
}

bool Reader::has(const std::string& name) {
  Loc l;
  return locate(name, &l);
}

std::vector<std::string> Reader::names() {
  std::lock_guard<std::mutex> g(mu_);
  rescan_locked();
  std::vector<std::string> out;
  for (auto& kv : where_) out.push_back(kv.first);
  std::sort(out.begin(), out.end());
  return out;
}

bool Reader::info(const std::string& name, Info* out) {
  Loc l;
  if (!locate(name, &l)) return false;
  const CamEntry& e = l.seg->hdr->cams[l.cam];
  out->owner_pid = l.seg->pid;
  out->pinned = e.pinned.load() != 0;
  out->ring_seq = e.ring_seq.load();
  out->bus_seq = e.bus_seq.load();
  out->published = l.seg->hdr->published.load();
  return true;
}

bool Reader::touch(const std::string& name, int key_frame_only) {
  Loc l;
  if (!locate(name, &l)) return false;
  Header* h = l.seg->hdr;
  CamEntry& e = h->cams[l.cam];
  if (key_frame_only >= 0) e.keyframe_only.store(key_frame_only ? 1u : 0u, std::memory_order_release);
  const i64 now = wall_ms();
  i64 cur = e.last_query_ms.load();
  while (cur < now && !e.last_query_ms.compare_exchange_weak(cur, now)) {
  }
  h->doorbell.fetch_add(1, std::memory_order_acq_rel);  // the pump forwards it to the decoder
  futex_wake(&h->doorbell);
  return true;
}

bool Reader::wait(const std::string& name, i64 after, int wait_ms, int key_frame_only, Ticket* t, bool touch,
                  const std::atomic<bool>* cancel) {
  Loc l;
  if (!locate(name, &l)) return false;
  Header* h = l.seg->hdr;
  CamEntry& e = h->cams[l.cam];
  if (touch) {
    if (key_frame_only >= 0) e.keyframe_only.store(key_frame_only ? 1u : 0u, std::memory_order_release);
    const i64 now = wall_ms();
    i64 cur = e.last_query_ms.load();
    while (cur < now && !e.last_query_ms.compare_exchange_weak(cur, now)) {
    }
  }
  const i64 rs = e.ring_seq.load(std::memory_order_acquire);
  if (rs < after) after = 0;  // the cursor belongs to an older ring (restarted owner / new camera)
  const i64 want = std::max(after + 1, rs);
  auto ready = [&] {
    return e.bus_seq.load(std::memory_order_acquire) >= want || !e.live.load(std::memory_order_acquire) ||
           e.gen.load(std::memory_order_acquire) != l.gen;
  };
  bool ok = ready();
  if (!ok) {
    e.waiters.fetch_add(1, std::memory_order_acq_rel);
    h->doorbell.fetch_add(1, std::memory_order_acq_rel);
    futex_wake(&h->doorbell);
    // wait_ms bounds the wait for a NEW frame; a frame the ring already holds only needs the
    // pump's DMA, which is given up to a second even when the caller does not wait (wait_ms 0)
    const i64 deadline = mono_ms() + std::max(std::max(0, wait_ms), rs > after ? 1000 : 0);
    for (;;) {
      const u32 p = e.pub.load(std::memory_order_acquire);
      if ((ok = ready())) break;
      const i64 left = deadline - mono_ms();
      if (left <= 0 || !pid_alive(l.seg->pid)) break;
      if (cancel && cancel->load(std::memory_order_acquire)) break;
      futex_wait(&e.pub, p, int(std::min<i64>(left, 100)));
    }
    e.waiters.fetch_sub(1, std::memory_order_acq_rel);
  } else {
    // the pump forwards the new last_query / mode to the decoder
    h->doorbell.fetch_add(1, std::memory_order_acq_rel);
    futex_wake(&h->doorbell);
  }
  if (!ok || !e.live.load(std::memory_order_acquire) || e.gen.load(std::memory_order_acquire) != l.gen) return false;
  t->seg = l.seg;
  t->cam = l.cam;
  t->gen = l.gen;
  t->after = after;
  t->cap = size_t(e.slot_cap.load(std::memory_order_acquire));
  return t->cap > 0;
}

i64 Reader::newest_seq(const Ticket& t) const {
  const Seg* seg = static_cast<const Seg*>(t.seg.get());
  const CamEntry& e = seg->hdr->cams[t.cam];
  return e.bus_seq.load(std::memory_order_acquire);
}

// The camera's data segment of generation dg, mapped once per reader (null: replaced meanwhile).
std::shared_ptr<void> Reader::data_map(const std::shared_ptr<Seg>& seg, int cam, u32 gen, u32 dg, u64 scap) {
  std::lock_guard<std::mutex> g(mu_);
  const std::string key = seg->path + "/" + std::to_string(cam);
  auto it = data_.find(key);
  if (it == data_.end() || it->second.data_gen != dg || it->second.cam_gen != gen) {
    if (it != data_.end()) data_.erase(it);  // the camera's older segment: unmapped
    const std::string path = seg->path + ".c" + std::to_string(cam) + ".g" + std::to_string(dg);
    auto m = std::make_shared<DataSeg>();
    m->bytes = size_t(scap) * kSlots;
    m->base = static_cast<const u8*>(map_file(path, m->bytes, false, false));
    if (!m->base) return nullptr;
    data_[key] = DataMap{seg->path, cam, dg, gen, m};
  }
  return data_[key].map;
}

std::shared_ptr<const Reader::Lease> Reader::lease(const Ticket& t) {
  auto seg = std::static_pointer_cast<Seg>(t.seg);
  CamEntry& e = seg->hdr->cams[t.cam];
  for (int attempt = 0; attempt < 8; ++attempt) {
    if (!e.live.load(std::memory_order_acquire) || e.gen.load(std::memory_order_acquire) != t.gen) return nullptr;
    const u32 dg = e.data_gen.load(std::memory_order_acquire);
    const u64 scap = e.slot_cap.load(std::memory_order_acquire);
    if (dg == 0 || scap == 0) return nullptr;
    std::shared_ptr<DataSeg> ds = std::static_pointer_cast<DataSeg>(data_map(seg, t.cam, t.gen, dg, scap));
    if (!ds) continue;
    const u32 k = e.newest.load(std::memory_order_acquire) % kSlots;
    SlotHdr& s = e.slots[k];
    s.leases.fetch_add(1, std::memory_order_seq_cst);
    const i64 now = mono_ms();
    i64 until = s.lease_until.load(std::memory_order_relaxed);
    while (until < now + kLeaseMs && !s.lease_until.compare_exchange_weak(until, now + kLeaseMs)) {
    }
    const u64 v = s.version.load(std::memory_order_seq_cst);
    const i64 sq = s.seq.load(std::memory_order_acquire);
    const u64 len = s.len.load(std::memory_order_acquire);
    if ((v & 1) || sq <= t.after || len == 0 || len > scap || e.data_gen.load(std::memory_order_acquire) != dg) {
      s.leases.fetch_sub(1, std::memory_order_acq_rel);
      if (!(v & 1) && sq <= t.after) return nullptr;
      continue;
    }
    // the lease object keeps both segments mapped and gives the slot back when dropped
    struct Held {
      Lease l;
      std::shared_ptr<Seg> seg;
      std::shared_ptr<DataSeg> ds;
      SlotHdr* s;
      ~Held() { s->leases.fetch_sub(1, std::memory_order_acq_rel); }
    };
    auto h = std::make_shared<Held>();
    h->l.data = ds->base + size_t(k) * scap;
    h->l.len = size_t(len);
    h->l.seq = sq;
    h->l.taken_ms = now;
    h->seg = seg;
    h->ds = ds;
    h->s = &s;
    leases_taken_.fetch_add(1);
    return std::shared_ptr<const Lease>(h, &h->l);
  }
  return nullptr;
}

size_t Reader::copy(const Ticket& t, u8* dst, size_t cap, i64* seq) {
  auto seg = std::static_pointer_cast<Seg>(t.seg);
  CamEntry& e = seg->hdr->cams[t.cam];
  for (int attempt = 0; attempt < 8; ++attempt) {
    if (!e.live.load(std::memory_order_acquire) || e.gen.load(std::memory_order_acquire) != t.gen) return 0;
    const u32 dg = e.data_gen.load(std::memory_order_acquire);
    const u64 scap = e.slot_cap.load(std::memory_order_acquire);
    if (dg == 0 || scap == 0) return 0;
    std::shared_ptr<DataSeg> ds = std::static_pointer_cast<DataSeg>(data_map(seg, t.cam, t.gen, dg, scap));
    if (!ds) continue;  // (replaced meanwhile)
    const u32 k = e.newest.load(std::memory_order_acquire);
    const SlotHdr& s = e.slots[k % kSlots];
    const u64 v1 = s.version.load(std::memory_order_acquire);
    if (v1 & 1) continue;
    const i64 sq = s.seq.load(std::memory_order_acquire);
    const u64 len = s.len.load(std::memory_order_acquire);
    if (sq <= t.after || len == 0 || len > cap || len > scap) {
      if (sq <= t.after) return 0;
      continue;
    }
    std::memcpy(dst, ds->base + size_t(k % kSlots) * scap, len);
    std::atomic_thread_fence(std::memory_order_acquire);
    if (s.version.load(std::memory_order_acquire) != v1 || e.data_gen.load(std::memory_order_acquire) != dg) continue;
    *seq = sq;
    return size_t(len);
  }
  return 0;
}

}  // namespace vep::bus
