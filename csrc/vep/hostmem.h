// Device-accessible host memory for ingest: a size-class pool of pinned (hipHostMalloc, mapped)
// blocks that access units are finalised into, and a registry translating host addresses inside
// such blocks to device addresses.
//
// Why: the native decoder references PCM samples *in place* in the received slice bytes. When
// those bytes already sit in pinned memory the worker's critical path does no host copy at all —
// a gather kernel on the copy stream pulls each slice straight over PCIe into the device staging
// buffer. The one host copy that remains (RTP reassembly -> pinned block) runs on the camera's
// own ingest thread, in parallel across cameras. Replaces the reference's
// ndarray/tobytes/SerializeToString/Redis copy chain (python/read_image.py:94-121).
#pragma once

#include <memory>
#include <mutex>

#include "common.h"

namespace vep::hostmem {

// Enable the pinned pool (called once a Worker owns a GPU; HIP must be initialised). Until
// then, and on CPU-only hosts, pinned_block() returns nullptr and AUs stay in pageable memory.
void enable_pool(size_t max_bytes = size_t(8) << 30);
bool pool_enabled();

// A block of at least n bytes from the pool (nullptr if disabled or over budget). The memory is
// returned to the pool when the last reference drops.
std::shared_ptr<u8> pinned_block(size_t n);

// Device address of [p, p + n) if the range lies inside a registered pinned region, else nullptr.
const u8* device_address(const u8* p, size_t n);

// Register / unregister externally allocated pinned memory (e.g. a staging buffer).
void register_range(const u8* host, size_t n, const u8* dev);
void unregister_range(const u8* host);

struct PoolStats {
  u64 chunks = 0, bytes_reserved = 0, blocks_live = 0, blocks_reused = 0, fallbacks = 0;
};
PoolStats pool_stats();

}  // namespace vep::hostmem
