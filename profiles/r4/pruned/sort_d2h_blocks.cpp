// On this image the runtime executes such copies as blit kernels
// (__amd_rocclr_copyBuffer, ~512 workgroups whose waves wait on PCIe): a
// large download then holds CU slots of the next map running beside it.
// g_d2h_blocks > 0 copies with our own kernel on that many workgroups instead.
static int g_d2h_blocks = 0;

int mr_d2h_set_blocks(int blocks) {
  if (blocks < 0 || blocks > 8192) return -1;
  g_d2h_blocks = blocks;
  return 0;
}

int mr_d2h_async(void* host_dst, const void* src, u64 nbytes, hipStream_t s) {
  if (nbytes == 0) return 0;
  if (g_d2h_blocks > 0) {
    void* dptr = nullptr;
    if (hipHostGetDevicePointer(&dptr, host_dst, 0) != hipSuccess || dptr == nullptr) dptr = host_dst;
    hipLaunchKernelGGL(copy_to_host_kernel, dim3(g_d2h_blocks), dim3(256), 0, s, (const u8*)src, (u8*)dptr,
                       (const long long*)nullptr, (u64)1, nbytes);
    return (int)hipGetLastError();
  }
  return (int)hipMemcpyAsync(host_dst, src, nbytes, hipMemcpyDeviceToHost, s);
}

