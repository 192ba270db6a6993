// streams.hip — streams restricted to a set of CUs (hipExtStreamCreateWithCUMask).
//
// A W > 1 iteration runs its post-map chain (compaction, pack, count
// exchange, receive-side insert, tail: ~30 short latency-bound launches) beside
// the next iteration's map, which fills every CU: each small launch then waits
// for CU slots behind the map's workgroups (the tail's sort passes ran 1.5-2x
// slower, profiles/r5/post/).  Stream priorities did not change that.  Giving
// the post-map stream a few CUs of its own and the map streams the rest keeps
// the two apart.
#include <hip/hip_runtime.h>
#include <cstdint>

extern "C" {

// CUs of the current device.
int mr_device_cus() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
  return n;
}

// A new stream on the current device whose kernels run on the CUs set in
// mask[0..nwords) (bit i of word w = CU 32 w + i); null on failure.
void* mr_stream_cumask(const uint32_t* mask, uint32_t nwords) {
  hipStream_t s = nullptr;
  if (hipExtStreamCreateWithCUMask(&s, nwords, mask) != hipSuccess) return nullptr;
  return (void*)s;
}

int mr_stream_destroy(void* s) { return (int)hipStreamDestroy((hipStream_t)s); }

}  // extern "C"
