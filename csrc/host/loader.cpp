// loader.cpp — native split loader: files (or byte ranges of files) read by a
// pool of threads straight into a caller-owned (pinned) host buffer.
//
// This is the host half of the reference's map input path: every map job
// opens its split file and reads it line by line (examples/WordCount/mapfn.lua:4,
// the WordCountBig taskfn lists 197 split files, examples/WordCountBig/taskfn.lua:6-10).
// Here a rank reads only the splits it owns, in parallel, with pread() into the
// pinned staging buffer the host->HBM copies read from, and publishes a
// per-split "ready" flag as soon as the split's last byte has landed so the
// copy of a chunk can start while later splits are still being read.
//
//   h = mrh_load_start(n, paths, file_off, len, dst_off, pad, dst, ready, nthreads, piece)
//       job i: read len[i] bytes of paths[i] from file_off[i] into dst + dst_off[i];
//       pad[i] != 0 writes '\n' at dst + dst_off[i] + len[i] (a split that does not
//       end in whitespace is terminated so no token straddles two splits).
//       Jobs larger than `piece` bytes are split into pieces read by different
//       threads.  ready[i] becomes 1 (release store) when job i is complete, -1 on
//       error.  Threads take pieces in job order, so early jobs finish first.
//   mrh_load_done(h)  -> number of complete jobs
//   mrh_load_wait(h)  -> 0, or -errno of the first failure; joins and frees h
//   mrh_drop_cache(path) -> posix_fadvise(DONTNEED): evict the file's clean pages
//       (a cold-read measurement without root)
#include <errno.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

struct Piece {
  int job;
  int64_t file_off, len, dst_off;
};

struct Load {
  std::vector<std::string> paths;
  std::vector<int64_t> len, dst_off;
  std::vector<int32_t> pad;
  std::vector<Piece> pieces;
  std::vector<std::atomic<int64_t>> remaining;  // pieces left per job
  uint8_t* dst = nullptr;
  int32_t* ready = nullptr;
  std::atomic<size_t> next{0};
  std::atomic<int> done{0};
  std::atomic<int> err{0};
  std::vector<std::thread> threads;

  explicit Load(int n) : remaining(n) {}

  void finish_job(int j) {
    if (pad[j]) dst[dst_off[j] + len[j]] = '\n';
    __atomic_store_n(&ready[j], 1, __ATOMIC_RELEASE);
    done.fetch_add(1, std::memory_order_release);
  }

  void fail(int j, int e) {
    int z = 0;
    err.compare_exchange_strong(z, -e);
    __atomic_store_n(&ready[j], -1, __ATOMIC_RELEASE);
  }

  void worker() {
    // one descriptor per (thread, file) run: pieces of one file are usually
    // consecutive in the queue
    int fd = -1, fd_job = -1;
    for (;;) {
      const size_t k = next.fetch_add(1, std::memory_order_relaxed);
      if (k >= pieces.size()) break;
      const Piece& p = pieces[k];
      if (p.len == 0) {
        if (remaining[p.job].fetch_sub(1) == 1) finish_job(p.job);
        continue;
      }
      if (fd_job < 0 || paths[fd_job] != paths[p.job]) {
        if (fd >= 0) close(fd);
        fd = open(paths[p.job].c_str(), O_RDONLY | O_CLOEXEC);
        fd_job = p.job;
        if (fd < 0) {
          fail(p.job, errno);
          fd_job = -1;
          continue;
        }
      }
      int64_t got = 0;
      int e = EIO;  // a short file reads 0 bytes before `len`
      while (got < p.len) {
        const ssize_t r = pread(fd, dst + p.dst_off + got, (size_t)(p.len - got), (off_t)(p.file_off + got));
        if (r < 0 && errno == EINTR) continue;
        if (r < 0) e = errno;
        if (r <= 0) break;
        got += r;
      }
      if (got != p.len) {
        fail(p.job, e);
        continue;
      }
      if (remaining[p.job].fetch_sub(1) == 1) finish_job(p.job);
    }
    if (fd >= 0) close(fd);
  }
};

}  // namespace

extern "C" {

void* mrh_load_start(int n, const char** paths, const int64_t* file_off, const int64_t* len, const int64_t* dst_off,
                     const int32_t* pad, uint8_t* dst, int32_t* ready, int nthreads, int64_t piece) {
  if (n < 0 || !dst || !ready) return nullptr;
  Load* L = new Load(n);
  L->dst = dst;
  L->ready = ready;
  if (piece <= 0) piece = 8 << 20;
  L->paths.reserve(n);
  for (int i = 0; i < n; ++i) {
    L->paths.emplace_back(paths[i]);
    L->len.push_back(len[i]);
    L->dst_off.push_back(dst_off[i]);
    L->pad.push_back(pad ? pad[i] : 0);
    ready[i] = 0;
    int64_t np = 0;
    for (int64_t o = 0; o < len[i] || (o == 0 && len[i] == 0); o += piece) {
      const int64_t l = len[i] - o < piece ? len[i] - o : piece;
      L->pieces.push_back(Piece{i, file_off[i] + o, l > 0 ? l : 0, dst_off[i] + o});
      ++np;
      if (len[i] == 0) break;
    }
    L->remaining[i].store(np);
  }
  if (nthreads <= 0) nthreads = 8;
  if ((size_t)nthreads > L->pieces.size()) nthreads = (int)L->pieces.size();
  if (nthreads < 1) nthreads = 1;
  for (int t = 0; t < nthreads; ++t) L->threads.emplace_back([L] { L->worker(); });
  return L;
}

int mrh_load_done(void* h) { return h ? static_cast<Load*>(h)->done.load(std::memory_order_acquire) : 0; }

int mrh_load_wait(void* h) {
  if (!h) return -EINVAL;
  Load* L = static_cast<Load*>(h);
  for (auto& t : L->threads) t.join();
  const int e = L->err.load();
  delete L;
  return e;
}

int mrh_drop_cache(const char* path) {
  const int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -errno;
  fdatasync(fd);
  const int r = posix_fadvise(fd, 0, 0, POSIX_FADV_DONTNEED);
  close(fd);
  return -r;
}

}  // extern "C"
