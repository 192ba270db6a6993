// sdma.hip — device -> pinned-host downloads on the SDMA copy engines.
//
// hipMemcpyAsync(DeviceToHost) into pinned memory runs, on this image's
// runtime, as a blit kernel (__amd_rocclr_copyBuffer) on the compute units:
// a large result download (the bigram job's ~575 MB per step) then competes
// with the next iteration's map for CUs and slows it 1.6-4x
// (profiles/r4/general/bigram_ab/).  The ROCr copy API between a GPU agent
// and the CPU agent uses the SDMA engines instead; the caller issues it once
// the producing kernels are done (their stream was waited on), and the copies
// of one batch complete together on one signal.  Any failure falls back to
// hipMemcpy (the caller's data is always produced).  mr_sdma_d2h_begin
// returns with the copies in flight, so the host can queue the next
// iteration's kernels while its results land (mr_sdma_wait before reading).
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <cstdint>
#include <mutex>

namespace {

std::mutex g_mu;
int g_state = 0;  // 0: not tried, 1: ready, -1: unavailable
hsa_agent_t g_cpu;

hsa_status_t find_cpu(hsa_agent_t a, void* data) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (t == HSA_DEVICE_TYPE_CPU) {
    *static_cast<hsa_agent_t*>(data) = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

bool ready() {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_state == 0) {
    g_state = -1;
    // the HIP runtime has initialised ROCr; this only takes a reference
    if (hsa_init() == HSA_STATUS_SUCCESS) {
      g_cpu.handle = 0;
      hsa_iterate_agents(find_cpu, &g_cpu);
      if (g_cpu.handle) g_state = 1;
    }
  }
  return g_state == 1;
}

bool gpu_owner(const void* p, hsa_agent_t* out) {
  hsa_amd_pointer_info_t info;
  info.size = sizeof(info);
  if (hsa_amd_pointer_info(const_cast<void*>(p), &info, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS) return false;
  if (info.type == HSA_EXT_POINTER_TYPE_UNKNOWN) return false;
  hsa_device_type_t t;
  if (hsa_agent_get_info(info.agentOwner, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_GPU)
    return false;
  *out = info.agentOwner;
  return true;
}

}  // namespace

extern "C" {

// 1 when the SDMA download path is usable in this process.
int mr_sdma_available() { return ready() ? 1 : 0; }

// Issue n downloads dsts[i] <- srcs[i] (sizes[i] bytes; device memory ->
// pinned host memory) on the SDMA engines, all completing on one signal, and
// return without waiting: > 0 = the batch's handle for mr_sdma_wait.  0 = the
// copies are done already (through hipMemcpy: SDMA unusable, or nothing to
// copy); -1 = a hipMemcpy fallback failed.  *fell_back = 1 when hipMemcpy ran.
uint64_t mr_sdma_d2h_begin(void* const* dsts, const void* const* srcs, const uint64_t* sizes, int n, int* fell_back) {
  *fell_back = 0;
  if (n <= 0) return 0;
  bool ok = ready();
  hsa_signal_t sig{0};
  int issued = 0;
  if (ok && hsa_signal_create(n, 0, nullptr, &sig) != HSA_STATUS_SUCCESS) ok = false;
  for (int i = 0; ok && i < n; ++i) {
    hsa_agent_t gpu;
    if (!sizes[i]) {
      hsa_signal_subtract_screlease(sig, 1);
      ++issued;
      continue;
    }
    if (!gpu_owner(srcs[i], &gpu) ||
        hsa_amd_memory_async_copy(dsts[i], g_cpu, srcs[i], gpu, sizes[i], 0, nullptr, sig) != HSA_STATUS_SUCCESS) {
      ok = false;
      break;
    }
    ++issued;
  }
  if (sig.handle) {
    hsa_signal_subtract_screlease(sig, n - issued);  // the copies never issued
    if (ok) return sig.handle;
    // a copy failed to issue: the issued ones must finish before hipMemcpy
    // rewrites their buffers
    hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
    hsa_signal_destroy(sig);
  }
  *fell_back = 1;
  for (int i = 0; i < n; ++i)
    if (sizes[i] && hipMemcpy(dsts[i], srcs[i], sizes[i], hipMemcpyDeviceToHost) != hipSuccess) return (uint64_t)-1;
  return 0;
}

// Wait for a batch of mr_sdma_d2h_begin and release its signal: 0, or -1
// when a copy reported an error (the signal went negative).
int mr_sdma_wait(uint64_t handle) {
  if (handle == 0) return 0;
  hsa_signal_t sig;
  sig.handle = handle;
  const hsa_signal_value_t v =
      hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
  hsa_signal_destroy(sig);
  return v < 0 ? -1 : 0;
}

// The blocking form: begin + wait.  Returns 0, 1 when the copies went
// through hipMemcpy instead (SDMA unusable), -1 on failure.
int mr_sdma_d2h(void* const* dsts, const void* const* srcs, const uint64_t* sizes, int n) {
  int fell_back = 0;
  const uint64_t h = mr_sdma_d2h_begin(dsts, srcs, sizes, n, &fell_back);
  if (h == (uint64_t)-1) return -1;
  if (fell_back) return 1;
  if (mr_sdma_wait(h) < 0) {  // a copy failed on the engine: redo them all
    for (int i = 0; i < n; ++i)
      if (sizes[i] && hipMemcpy(dsts[i], srcs[i], sizes[i], hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return 1;
  }
  return 0;
}

}  // extern "C"
