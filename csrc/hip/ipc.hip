// ipc.hip — device-resident intermediate files shared between worker
// processes (the "hbm" storage of runtime/hbm_store.py).
//
// The reference's storages all work across worker processes and hosts:
// GridFS through mongod, "shared" through NFS, "sshfs" through scp
// (/root/reference/mapreduce/fs.lua:185-208); a reduce job reads the map files
// any worker wrote (job.lua:253-260).  On one MI355X node the natural store is
// HBM itself: a map worker keeps its partition files in an arena of device
// memory it exports with hipIpcGetMemHandle; the coordinator's file entry holds
// the handle and the file's place in the arena; a reducer on any GPU of the
// node maps the arena (hipIpcOpenMemHandle) and pulls the files it needs with
// ONE gather-copy launch over xGMI (or inside the GPU) into its own buffer, where
// ONE decode launch turns the columnar files (runtime/codec.py MRC1) into the
// reduce table's input columns.  No byte of the intermediate data goes through
// host memory or the coordinator's socket.
//
//   mr_ipc_alloc / mr_ipc_free        hipMalloc'd arena chunks (exportable)
//   mr_ipc_handle                     the 64-byte hipIpcMemHandle_t of a chunk
//   mr_ipc_open / mr_ipc_close        a peer's chunk in this process
//   mr_gather_copy                    n (src, dst, len) copies in one launch
//   mr_mrc1_decode                    MRC1 files in one buffer -> hi, lo, val, rep
#include <hip/hip_runtime.h>
#include <cstring>
#include "mr_common.h"

namespace mr {

// One workgroup per copy run of up to GC_CHUNK bytes: 16-byte vector loads and
// stores when source, destination and length allow, else bytes.  Sources may be
// peer memory (an IPC-mapped chunk of another GPU: the loads cross xGMI).
constexpr int GC_T = 256;
constexpr u64 GC_CHUNK = 1ull << 18;

__global__ void __launch_bounds__(GC_T) gather_copy_kernel(const u64* __restrict__ srcs, const u64* __restrict__ dsts,
                                                           const u64* __restrict__ lens,
                                                           const u64* __restrict__ chunk_start, u32 n) {
  // chunk_start[i] = first chunk of copy i (prefix over ceil(len / GC_CHUNK))
  const u64 c = blockIdx.x;
  u32 lo = 0, hi = n;
  while (hi - lo > 1) {
    const u32 mid = (lo + hi) / 2;
    if (chunk_start[mid] <= c) lo = mid; else hi = mid;
  }
  const u32 i = lo;
  const u64 off = (c - chunk_start[i]) * GC_CHUNK;
  const u64 len = lens[i];
  if (off >= len) return;
  const u64 m = len - off < GC_CHUNK ? len - off : GC_CHUNK;
  const u8* s = reinterpret_cast<const u8*>(srcs[i]) + off;
  u8* d = reinterpret_cast<u8*>(dsts[i]) + off;
  if ((((uintptr_t)s ^ (uintptr_t)d) & 15) == 0) {
    // same offset mod 16 on both sides: a byte head up to the next 16-byte
    // boundary, then 16-byte vectors, then a byte tail
    u64 head = (16 - ((uintptr_t)s & 15)) & 15;
    if (head > m) head = m;
    if (threadIdx.x < head) d[threadIdx.x] = s[threadIdx.x];
    const u64 n16 = (m - head) / 16;
    const uint4* s4 = reinterpret_cast<const uint4*>(s + head);
    uint4* d4 = reinterpret_cast<uint4*>(d + head);
    for (u64 k = threadIdx.x; k < n16; k += GC_T) d4[k] = s4[k];
    for (u64 k = head + n16 * 16 + threadIdx.x; k < m; k += GC_T) d[k] = s[k];
  } else {
    for (u64 k = threadIdx.x; k < m; k += GC_T) d[k] = s[k];
  }
}

// MRC1 file j at byte base[j] of buf (base[j] % 8 == 4, so its 8-byte columns
// after the 20-byte header are aligned): rows rstart[j] .. rstart[j+1] of the
// output.  Layout (codec.encode_columnar): "MRC1" n nb | hi[n] lo[n] val[n]
// key_off[n+1] | key bytes.  rep = (byte offset of the key in buf) << 24 | len,
// so buf itself is the key-byte source of the reduce table.
constexpr int DC_T = 256;
__global__ void __launch_bounds__(DC_T) mrc1_decode_kernel(const u8* __restrict__ buf, const u64* __restrict__ base,
                                                           const u64* __restrict__ rstart, u32 nfiles, u64 nrows,
                                                           u64* __restrict__ o_hi, u64* __restrict__ o_lo,
                                                           long long* __restrict__ o_val, u64* __restrict__ o_rep) {
  const u64 r = (u64)blockIdx.x * DC_T + threadIdx.x;
  if (r >= nrows) return;
  u32 lo = 0, hi = nfiles;
  while (hi - lo > 1) {
    const u32 mid = (lo + hi) / 2;
    if (rstart[mid] <= r) lo = mid; else hi = mid;
  }
  const u64 n = rstart[lo + 1] - rstart[lo];
  const u64 k = r - rstart[lo];
  const u64 b = base[lo] + 20;
  const u64* col = reinterpret_cast<const u64*>(buf + b);
  const long long* koff = reinterpret_cast<const long long*>(col + 3 * n);
  const u64 kb = b + 8 * (4 * n + 1);
  const long long o = koff[k];
  o_hi[r] = col[k];
  o_lo[r] = col[n + k];
  o_val[r] = (long long)col[2 * n + k];
  o_rep[r] = make_rep(kb + (u64)o, (u64)(koff[k + 1] - o));
}

}  // namespace mr

using namespace mr;

extern "C" {

int mr_ipc_alloc(unsigned long long nbytes, void** out) {
  *out = nullptr;
  return (int)hipMalloc(out, nbytes ? nbytes : 1);
}

int mr_ipc_free(void* p) { return p ? (int)hipFree(p) : 0; }

int mr_ipc_handle(void* p, void* out64) {
  hipIpcMemHandle_t h;
  const hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess) return (int)e;
  static_assert(sizeof(h) == 64, "hipIpcMemHandle_t is 64 bytes");
  std::memcpy(out64, &h, sizeof(h));
  return 0;
}

int mr_ipc_open(const void* handle64, void** out) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle64, sizeof(h));
  *out = nullptr;
  return (int)hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess);
}

int mr_ipc_close(void* p) { return p ? (int)hipIpcCloseMemHandle(p) : 0; }

// table = device u64 [4 * n]: srcs | dsts | lens | chunk_start (the launch's
// copy list, uploaded by the caller); nchunks = chunk_start[n - 1] + chunks of
// the last copy
int mr_gather_copy(const void* table, unsigned n, unsigned long long nchunks, hipStream_t s) {
  if (n == 0 || nchunks == 0) return 0;
  const u64* t = static_cast<const u64*>(table);
  hipLaunchKernelGGL(gather_copy_kernel, dim3((unsigned)nchunks), dim3(GC_T), 0, s, t, t + n, t + 2 * n, t + 3 * n, n);
  return (int)hipGetLastError();
}

unsigned long long mr_gather_copy_chunk() { return GC_CHUNK; }

// meta = device u64 [2 * nfiles + 1]: base[nfiles] | rstart[nfiles + 1]
int mr_mrc1_decode(const void* buf, const void* meta, unsigned nfiles, unsigned long long nrows, void* hi, void* lo,
                   void* val, void* rep, hipStream_t s) {
  if (nrows == 0 || nfiles == 0) return 0;
  const u64* m = static_cast<const u64*>(meta);
  const u64 g = (nrows + DC_T - 1) / DC_T;
  hipLaunchKernelGGL(mrc1_decode_kernel, dim3((unsigned)g), dim3(DC_T), 0, s, (const u8*)buf, m, m + nfiles, nfiles,
                     nrows, (u64*)hi, (u64*)lo, (long long*)val, (u64*)rep);
  return (int)hipGetLastError();
}

}  // extern "C"
