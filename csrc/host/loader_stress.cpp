// loader_stress.cpp — multi-threaded stress client of the native split loader
// (loader.cpp), built with it under ThreadSanitizer / AddressSanitizer +
// UndefinedBehaviorSanitizer by tests/test_native_sanitizers.py.
//
// Writes `nfiles` files of random sizes (some empty, some not ending in a
// newline), loads them with many threads and small pieces (every job split
// over several threads) into one buffer, and meanwhile a consumer thread
// polls the per-job ready flags with acquire loads and checks every job the
// moment it is published — the way the engine starts a chunk's host->HBM copy
// while later splits are still being read.  One job names a missing file (the
// failure path).  Exit 0 and "loader_stress ok" when every byte and pad is
// right and the error is reported.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <string>
#include <thread>
#include <vector>

extern "C" {
void* mrh_load_start(int n, const char** paths, const int64_t* file_off, const int64_t* len, const int64_t* dst_off,
                     const int32_t* pad, uint8_t* dst, int32_t* ready, int nthreads, int64_t piece);
int mrh_load_done(void* h);
int mrh_load_wait(void* h);
}

int main(int argc, char** argv) {
  const int nfiles = argc > 1 ? atoi(argv[1]) : 64;
  const int nthreads = argc > 2 ? atoi(argv[2]) : 16;
  const int rounds = argc > 3 ? atoi(argv[3]) : 3;
  char dir[] = "/tmp/loader_stress_XXXXXX";
  if (!mkdtemp(dir)) return 2;
  srand(12345);
  std::vector<std::string> names;
  std::vector<std::string> content;
  for (int i = 0; i < nfiles; ++i) {
    const int64_t n = (i % 9 == 0) ? 0 : (rand() % 200000);
    std::string s(n, '\0');
    for (int64_t k = 0; k < n; ++k) s[k] = (char)(rand() & 0xFF);
    if (n && i % 3 == 0) s[n - 1] = '\n';
    std::string p = std::string(dir) + "/f" + std::to_string(i);
    FILE* f = fopen(p.c_str(), "wb");
    if (!f) return 2;
    fwrite(s.data(), 1, s.size(), f);
    fclose(f);
    names.push_back(p);
    content.push_back(s);
  }
  names.push_back(std::string(dir) + "/missing");
  content.push_back(std::string(10, 'x'));
  const int n = (int)names.size();
  int bad = 0;
  for (int round = 0; round < rounds; ++round) {
    std::vector<const char*> paths;
    std::vector<int64_t> off(n, 0), len(n), doff(n);
    std::vector<int32_t> pad(n), ready(n, 0);
    int64_t total = 0;
    for (int i = 0; i < n; ++i) {
      paths.push_back(names[i].c_str());
      len[i] = (int64_t)content[i].size();
      pad[i] = (len[i] == 0 || content[i].back() != '\n') ? 1 : 0;
      doff[i] = total;
      total += len[i] + pad[i];
    }
    std::vector<uint8_t> buf(total + 1, 0xAB);
    void* h = mrh_load_start(n, paths.data(), off.data(), len.data(), doff.data(), pad.data(), buf.data(),
                             ready.data(), nthreads, 4096 << (round % 3));
    if (!h) return 3;
    std::vector<char> seen(n, 0);
    int checked = 0;
    std::thread consumer([&] {
      int spins = 0;
      while (checked < n - 1 && spins < 200000000) {
        ++spins;
        for (int i = 0; i < n; ++i) {
          if (seen[i]) continue;
          const int r = __atomic_load_n(&ready[i], __ATOMIC_ACQUIRE);
          if (r == 0) continue;
          seen[i] = 1;
          if (r < 0) {
            if (i != n - 1) ++bad;
            continue;
          }
          ++checked;
          if (memcmp(buf.data() + doff[i], content[i].data(), len[i]) != 0) ++bad;
          if (pad[i] && buf[doff[i] + len[i]] != '\n') ++bad;
        }
      }
    });
    const int e = mrh_load_wait(h);
    consumer.join();
    if (e == 0) ++bad;  // the missing file must be reported
    if (checked != n - 1) ++bad;
  }
  for (auto& p : names) unlink(p.c_str());
  rmdir(dir);
  if (bad) {
    printf("loader_stress FAILED: %d\n", bad);
    return 1;
  }
  printf("loader_stress ok\n");
  return 0;
}
