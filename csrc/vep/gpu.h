// gfx950 device layer: memory, streams and the batched HIP kernels of the data plane.
//
// Kernels (gpu_kernels.hip):
//  * decode_convert — fused I_PCM macroblock reconstruction into the per-camera NV12 reference
//    surface + BT.601 NV12->BGR24 conversion into the camera's HBM ring slot. One launch per
//    worker step covers every camera of the GPU (block -> (camera, 8x2-MB tile)).
//    Replaces libavcodec reconstruction + libswscale (read_image.py:87,94).
//  * letterbox — NV12 surface -> letterboxed model input (HWC u8 and/or normalised CHW
//    fp16/bf16/fp32), batched over cameras.
#pragma once

#include <hip/hip_runtime.h>

#include "common.h"

namespace vep::gpu {

// Device-side view of the descriptors' buffer pointers in the kernel sources (which define
// VEP_KERNEL_SOURCE): the global address space. Kernels then issue global_load / global_store
// (counted by vmcnt only) instead of flat accesses, which also count against lgkmcnt and so tie
// every LDS or scalar-load wait to outstanding global traffic. Same size and layout as the
// plain pointers the host code fills in.
#if defined(__HIP_DEVICE_COMPILE__) && defined(VEP_KERNEL_SOURCE)
#define VEP_DEV __attribute__((address_space(1)))
#else
#define VEP_DEV
#endif

#define VEP_HIP(expr)                                                                    \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      throw ::vep::Error(std::string("HIP error ") + hipGetErrorString(_e) + " at " +     \
                         __FILE__ + ":" + std::to_string(__LINE__) + ": " #expr);        \
  } while (0)

int device_count();  // 0 when no GPU / no driver
bool rocdecode_available();  // VCN backend library present (backend.cpp)

// One camera-frame of a batched decode_convert launch (lives in device memory).
struct DecodeDesc {
  VEP_DEV u8* y;              // NV12 luma plane, pitch = wmbs*16
  VEP_DEV u8* uv;             // NV12 interleaved chroma plane, pitch = wmbs*16
  VEP_DEV u8* bgr;            // output slot: out_h x out_w x 3 (packed BGR24); may be null
  // Coded-MB bitmask (bit mb of word mb/32) + exclusive per-word popcount prefix: the payload
  // slot of a coded MB is prefix[w] + popc(mask[w] & below(mb)), slots in raster order.
  // null mask = no update (pure conversion). 2 bits/MB of H2D instead of a 32-bit map.
  const VEP_DEV u32* mask;
  const VEP_DEV u32* prefix;
  const VEP_DEV u32* offsets;  // per coded MB (raster order): byte offset of its 384 samples in payload
  const VEP_DEV u8* payload;   // the slices' bytes as received (samples read in place, unaligned)
  const VEP_DEV u64* ptrs;     // direct mode (non-null): per coded MB, device address of its samples in
                       // pinned host memory — read over PCIe; offsets/payload unused
  i32 wmbs, hmbs;
  i32 out_w, out_h;
  i32 crop_left, crop_top;
  i32 tile_begin;     // exclusive prefix sum of tiles over the batch
  i32 tiles_x;
  // Speculatively placed blocks (PictureInfo::spec_lo/hi): payload slots [chk_lo, chk_hi) must
  // be preceded by the 2 header bytes chk_pat (little-endian); a mismatch sets *err (pinned
  // host memory) and the worker drops the frame.
  i32 chk_lo, chk_hi;
  u32 chk_pat;
  VEP_DEV u32* err;
};
constexpr int kTileMbW = 8, kTileMbH = 2;  // 256 threads: 32 pixel rows x 8 MB columns
inline int tiles_for(int wmbs, int hmbs) {
  return ((wmbs + kTileMbW - 1) / kTileMbW) * ((hmbs + kTileMbH - 1) / kTileMbH);
}

void launch_decode_convert(const DecodeDesc* d_descs, int n, int total_tiles, hipStream_t s);
// Single-frame variant: descriptor passed by value (op API on caller-owned buffers).
void launch_decode_convert_one(const DecodeDesc& d, hipStream_t s);

// Gather: copy byte ranges from device-accessible (pinned, mapped) host memory into device
// memory over PCIe — one workgroup per chunk, 16-byte loads per lane. Replaces a host memcpy
// into staging + SDMA copy when the slice bytes already live in the pinned ingest pool.
struct GatherChunk {
  const VEP_DEV u8* src;  // device address of pinned host memory (any alignment)
  VEP_DEV u8* dst;        // device memory, 16-byte aligned
  u32 len;
  u32 pad;
};
constexpr u32 kGatherChunk = 32u << 10;
void launch_gather(const GatherChunk* d_chunks, int n, hipStream_t s);

// ---- general H.265 reconstruction (gpu_hevc.hip; records from hevc::Decoder, hevc_kern.h) ----
// One picture of a batched reconstruction round (device memory). DPB slot k of the camera
// lives at y + k * slot_y / uv + k * slot_uv (NV12, pitch = `stride` samples; slot sizes in
// bytes: Main10 pictures have u16 samples).
constexpr int kHevcWide = 16;
struct HevcDesc {
  VEP_DEV u8* y;
  VEP_DEV u8* uv;
  u64 slot_y, slot_uv;
  i32 stride, width, height;
  i32 log2ctb, wctb, hctb;
  i32 target;
  i32 cb_qp_offset, cr_qp_offset;
  i32 flags;             // bit 0 deblock, bit 1 SAO, bit 2 samples not loop-filtered (pcm_map),
                         // bit 3 SAO does not cross tile boundaries, bit 4 (kHevcWide) u16 samples
  i32 bd_y, bd_c;        // sample bit depths (8; Main10: up to 10, with kHevcWide)
  const VEP_DEV void* pus;       // hevc::GpuPu[npu]
  const VEP_DEV void* tus;       // hevc::GpuTu (level-sorted)
  const VEP_DEV i16* coefs;
  const VEP_DEV u8* pcm;
  const VEP_DEV u8* bs_v;
  const VEP_DEV u8* bs_h;
  const VEP_DEV signed char* qp;
  const VEP_DEV u8* pcm_map;
  const VEP_DEV u16* ctb_slice;
  const VEP_DEV void* slices;    // hevc::GpuSlice
  const VEP_DEV void* sao;       // hevc::GpuSao per CTB
  VEP_DEV u8* sao_y;             // device scratch: the deblocked picture (SAO input)
  VEP_DEV u8* sao_uv;
  const VEP_DEV void* wp;        // hevc::GpuWp (explicit weighted prediction, GpuPu::wp - 1)
  const VEP_DEV u16* ctb_tile;   // tile id per CTB
  VEP_DEV u32* err;              // the job's error word (bit 1: a dependency wait timed out)
  // Intra edge exchange (hevc_tu_queue_kernel): the camera's words, tagged with this round's
  // epoch, holding the right column / bottom row samples of every intra transform block.
  VEP_DEV u64* xg;
  i32 xg_h;              // coded height of the exchange's luma plane (width = stride)
  u32 epoch;             // tag of this round's words (never 0)
  i32 npu, pu_begin;     // exclusive prefix of PUs over the round
  i32 blk_begin;         // exclusive prefix of 4x4 blocks over the round
  // Polling backoff of a wave waiting on an edge word: it sleeps 256 cycles, then twice as long
  // after every miss, up to nap_max x 256 cycles (1: a fixed 256-cycle poll). Waves far ahead of
  // the wavefront then stop loading L2 with polls the producers' stores compete with.
  u32 nap_max;
  u32 pad_;
};
// Exchange words of a stride x h picture: luma columns (x % 4 == 3) and rows (y % 4 == 3), then
// the same for Cb and Cr. 3/4 word per luma sample.
inline size_t hevc_xg_words(int stride, int h) { return size_t(stride) * size_t(h) * 3 / 4; }
// Transform blocks tus[first .. first + count) of descs[desc], at tickets begin .. begin + count
// of their launch (intra queue: level-major, so a block's producers hold lower tickets).
struct HevcTuRange {
  i32 desc, first, count, begin;
};
// Motion compensation of every prediction block of the round (one workgroup per block).
void launch_hevc_mc(const HevcDesc* d_descs, int n, int total_pus, hipStream_t s);
// Independent transform blocks (level 0: inter residual + PCM; or the blocks of one intra level
// at tickets base .. base + count of the queue's ranges), one wave per block.
void launch_hevc_tu(const HevcDesc* d_descs, const HevcTuRange* d_ranges, int nranges, int base, int count,
                    hipStream_t s);
// Intra transform blocks at tickets base .. base + count (every intra level of the round, or a
// window of consecutive levels) in ONE launch: waves take tickets in level order from ctr[0]
// (zero at launch) — persistent waves until the queue is empty, or (windows) one ticket per wave
// — so every block a wave waits on was claimed by a running wave, whatever the dispatch order.
// A block reads the reference samples other intra blocks of the round write (GpuTu::pend) from
// their epoch-tagged edge words (HevcDesc::xg), polled until current, and publishes its own
// right column / bottom row the same way.
void launch_hevc_tu_queue(const HevcDesc* d_descs, const HevcTuRange* d_ranges, int nranges, int base, int count,
                          u32* ctr, bool persistent, hipStream_t s);
// Intra transform blocks, one workgroup per picture: d_pics[k] = {desc, first, count} names
// picture k's intra blocks tus[first .. first + count) (level-major); the workgroup's waves take
// them in order from an LDS counter, so every dependency wait stays inside one workgroup.
void launch_hevc_tu_pics(const HevcDesc* d_descs, const HevcTuRange* d_pics, int npics, hipStream_t s);
// Deblocking of every vertical (dir 0) or horizontal (dir 1) edge of the round, one thread per
// 4-line edge segment; then SAO (copy of the deblocked picture, one thread per sample).
void launch_hevc_deblock(const HevcDesc* d_descs, int n, int total_blocks, int dir, hipStream_t s);
void launch_hevc_sao(const HevcDesc* d_descs, int n, int total_blocks, hipStream_t s);
// Main10 output: u16 NV12 planes (n luma samples, n / 2 chroma) -> 8-bit NV12 (round to nearest,
// saturating), the form the BGR24 conversion and the letterbox read.
// 8-bit NV12 copy of a published slot (w x h luma): samples above 8 bits rounded to nearest
// (bd > 8: u16 planes), 4:2:2 chroma rows averaged in pairs (cf 2: an NV16 chroma plane of h rows)
// — the same result as narrow_surface (codec.h).
void launch_narrow(const void* y, const void* uv, u8* y8, u8* uv8, int w, int h, int bd, int cf, hipStream_t s);
// H.264 field pairs (frame slot in field-separated layout: top field rows, then bottom) -> the
// interleaved 8-bit NV12 frames (pitch bytes per row, `height` luma rows), one launch for the
// `n` descriptors of a batch (grid y = descriptor).
struct WeaveDesc {
  const VEP_DEV u8* y;
  const VEP_DEV u8* uv;
  VEP_DEV u8* y8;
  VEP_DEV u8* uv8;
  i32 pitch, height;
};
void launch_weave(const WeaveDesc* d_descs, int n, int max_pitch, int max_height, hipStream_t s);

// ---- general H.264 reconstruction (gpu_avc.hip; records from avc::Decoder, avc.h) ----------
// One picture of a batched reconstruction round (device memory). DPB slot k of the camera
// lives at y + k * slot_y / uv + k * slot_uv (NV12, pitch = wmbs * 16).
struct AvcDesc {
  const VEP_DEV void* mbs;     // avc::MbRec[wmbs * hmbs]
  const VEP_DEV i16* coefs;    // dequantised 4x4 blocks (16 x i16) / I_PCM samples
  const VEP_DEV i16* mvs;      // 32 x i16 per list per inter MB
  const VEP_DEV void* wps;     // avc::WpEntry pool (weighted prediction)
  VEP_DEV u8* y;
  VEP_DEV u8* uv;
  u64 slot_y, slot_uv;
  i32 wmbs, hmbs;
  i32 target;          // DPB slot reconstructed into
  i32 constrained;     // constrained_intra_pred_flag
  i32 mb_begin;        // exclusive prefix of MBs over the round (inter kernel block -> picture)
  i32 field;           // 0 frame; 1 / 2 top / bottom field picture (slots are fields, parity = slot & 1)
  VEP_DEV u32* err;            // pinned flag: wavefront timeout (frame dropped)
  VEP_DEV void* dbk;           // device scratch: AvcDbkInfo[wmbs * hmbs] (avc_bs_kernel -> deblock)
  VEP_DEV i16* res;            // device scratch: kAvcResSamples per intra MB with residual (MbRec::res
                       // slot; avc_inter_kernel -> avc_intra_kernel)
  VEP_DEV u64* prof;           // optional (VEP_AVC_PROF=1): kAvcProfSlots clock64() phase accumulators
  i32 bd;              // sample bit depth: 8 (u8 surfaces), 9 / 10 (High 10: u16 surfaces,
                       // slot_y / slot_uv in bytes; intra + deblocking in avc_hbd_kernel)
  i32 qp_bias, qpc_bias;  // MbRec::qp / qpc bias (QpBdOffsetY / C)
  i32 cf;              // chroma format: 1 (or 0: grey chroma) 4:2:0, 2 = 4:2:2 (NV16 slots; intra +
                       // deblocking in avc_hbd_kernel)
  // pool sizes (i16 coefficients, intra residual slots): the High 10 / 4:2:2 paths bound-check
  // every picture / pool access against them and report a violation in *err (bits 8..15)
  // instead of touching memory outside
  u32 ncoef, nres;
  i32 intra_mbs;       // intra MBs of the picture (avc_hbd_kernel skips its intra pass without)
  i32 deblock;         // any MB filtered (avc_hbd_kernel skips its loop-filter pass without)
  VEP_DEV u64* xg;             // device scratch: exchange between the wavefront workgroups, kAvcXgWords
                       // tagged words per MB of every workgroup's last row (intra wavefront:
                       // words 0..7, zeroed by avc_inter_kernel; deblocking: all, zeroed by
                       // avc_bs_kernel)
};
// Phase accumulators of the wavefront kernels (summed over waves): intra wait / load / luma /
// chroma / store+publish / MBs, deblock wait / load / filter / store+publish / MBs.
constexpr int kAvcProfSlots = 20;  // + [11] intra residual pass, [12..15] avc_hbd_kernel: intra
                                   // pass / loop-filter pass / barrier cycles (per workgroup),
                                   // pictures; [16..19] its loop filter per MB (wave 0): tile
                                   // load / edges / store cycles, MBs
// Residual samples of one intra MB: 256 luma (raster) + 2 x 64 chroma, as i16.
constexpr int kAvcResSamples = 512;  // slot stride: 256 luma + 2 x 64 chroma (4:2:2: 2 x 128)
// Per-MB loop-filter inputs, computed in parallel ahead of the deblocking wavefront.
struct AvcDbkInfo {
  u32 bs[4];      // 32 x 4-bit bS: nibble dir * 16 + edge * 4 + segment (0 = edge not filtered)
  u8 alpha[9], beta[9];  // [left, top, internal] for luma, Cb, Cr (component * 3 + edge kind)
  u8 tc0[9][3];   // tC0 for bS 1..3, same order
  u8 any;         // any bS != 0
  u8 pad[1];
};
static_assert(sizeof(AvcDbkInfo) == 64, "AvcDbkInfo layout");
// The deblocking wavefront runs kAvcDbkWgRows MB rows per workgroup (two per wave64), several
// workgroups per picture; a workgroup's last row hands its final bottom samples to the next
// workgroup through `xg`: 16 luma + 8 NV12 chroma u32 words per MB, each tagged (high half) with
// 2 once final (1 = columns 12..15 still to be filtered by the next MB's left edge).
constexpr int kAvcDbkWgRows = 8;
constexpr int kAvcXgWords = 24;
inline int avc_dbk_groups(int hmbs) { return (hmbs + kAvcDbkWgRows - 1) / kAvcDbkWgRows; }
inline size_t avc_xg_bytes(int wmbs, int hmbs) {
  return size_t(avc_dbk_groups(hmbs) - 1) * size_t(wmbs) * kAvcXgWords * sizeof(u64);
}
constexpr int kAvcMaxRows = 512;  // MB rows per picture the wavefront kernels support (8K)
constexpr int kAvcMaxCols = 512;  // MB columns
// Inter / skip / I_PCM macroblocks of every picture of the round (and intra MBs' residuals): one
// wave64 per MB, four per workgroup.
void launch_avc_inter(const AvcDesc* d_descs, int n, int total_mbs, hipStream_t s);
// Intra 4x4 / 16x16 macroblocks in a wavefront: avc_dbk_groups(hmbs) workgroups of
// kAvcDbkWgRows wave64s (one row each) per picture; rows synchronised through LDS counters
// inside a workgroup and tagged exchange words (AvcDesc::xg) between workgroups.
void launch_avc_intra(const AvcDesc* d_descs, int n, int max_hmbs, hipStream_t s);
// Boundary strengths + edge thresholds of every MB of the round (fully parallel), then the
// deblocking wavefront over them: avc_dbk_groups(hmbs) workgroups of kAvcDbkWgRows / 2 wave64s
// per picture, spread over the XCDs picture-wise (a picture's workgroups share one L2).
void launch_avc_bs(const AvcDesc* d_descs, int n, int total_mbs, hipStream_t s);
// packed: bit 0 vertical edges with word / half-word LDS accesses (VEP_DBK_PACKED=0: a byte per
// sample); bit 1 a wave sync after every edge instead of one per direction (VEP_DBK_SYNC=1)
void launch_avc_deblock(const AvcDesc* d_descs, int n, int max_hmbs, hipStream_t s, int packed = 1);
// High 10 pictures of the round (AvcDesc::bd > 8; the 8-bit wavefronts skip them): intra
// prediction, then (dbk: after launch_avc_bs) the loop filter. gpu_avc_hbd.hip
// variants: bit 0 High 10 4:2:0, bit 1 8-bit 4:2:2, bit 2 High 10 4:2:2 pictures present
void launch_avc_hbd(const AvcDesc* d_descs, int n, bool intra, bool dbk, int variants, hipStream_t s);

enum ChwDtype : int { kChwNone = 0, kChwF16 = 1, kChwBF16 = 2, kChwF32 = 3 };

struct LetterboxDesc {
  const VEP_DEV u8* y;
  const VEP_DEV u8* uv;
  i32 pitch;
  i32 src_w, src_h, crop_left, crop_top;
  VEP_DEV u8* out_hwc;      // S*S*3 BGR u8, or null
  VEP_DEV void* out_chw;    // 3*S*S RGB normalised, or null
  i32 nw, nh, pad_x, pad_y;
  float rx, ry;     // src/dst scale per axis
};
enum LetterboxFormat : int {
  kLbBGR = 0,   // out_hwc = S*S*3 packed BGR (+ optional normalised CHW)
  kLbNV12 = 1,  // out_hwc = S*S*3/2 NV12 (Y plane then interleaved UV): half the bytes on xGMI
};
struct LetterboxParams {
  i32 size;          // S
  i32 chw_dtype;     // ChwDtype
  float mean[3];     // RGB
  float inv_std[3];  // RGB
  u8 pad_value;
  i32 format = kLbBGR;
};
// even = true keeps the fitted size and padding on chroma-sample boundaries (NV12 output)
void fill_letterbox_geometry(LetterboxDesc& d, int size, bool even = false);
inline size_t letterbox_bytes(int size, int format) {
  return format == kLbNV12 ? size_t(size) * size * 3 / 2 : size_t(size) * size * 3;
}
// Consumer side: NV12 letterboxed batch [n][S*S*3/2] -> normalised RGB CHW [n][3][S][S].
void launch_nv12_to_chw(const u8* in, void* out, int n, int size, int chw_dtype,
                        const float mean[3], const float inv_std[3], hipStream_t s);
void launch_letterbox(const LetterboxDesc* d_descs, int n, const LetterboxParams& p,
                      hipStream_t s);
void launch_letterbox_one(const LetterboxDesc& d, const LetterboxParams& p, hipStream_t s);

}  // namespace vep::gpu
