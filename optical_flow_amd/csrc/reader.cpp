// Asynchronous KITTI batch reader (SURVEY.md §8 f row 1), the native counterpart of
// data_reader.py's AsyncReader (data_reader.py:81-124) + read_batch / read_item (:35-64).
//
// Reference: a multiprocessing.Pool of `nworkers` processes; each task decodes one whole
// batch with cv2 (imread -> resize -> /255 -> -mean) into a float32 (B,H,W,6) numpy array
// and puts it on a shared Queue, so batches arrive in completion order.  Here:
//   - worker THREADS decode PNGs (png_codec.cpp) image by image, straight into a pinned
//     host "slot" holding one batch of raw 8-bit BGR frames at their native size;
//   - of_reader_next() hands slots out strictly in submission order (deterministic), copies
//     the raw bytes to HBM on the caller's stream (8-bit frames: 1.4 MB per KITTI frame
//     instead of 2.4 MB of float32 at 384x512) and launches of_preprocess_pairs (the
//     resize + normalise + pair packing kernel, image_ops.hip) on that same stream;
//   - a slot is refilled with the next batch as soon as it is handed out; its workers first
//     wait on the event recorded after the slot's host->device copy.
// Batch bookkeeping follows add_fetch_task (:110-119): `nbatches = npairs / batch` (the
// remainder is dropped), pairs are taken in shuffled order, the order is reshuffled when the
// last batch of an epoch has been submitted, and each item is swapped with p = 0.5
// (read_item :46-51).  The reference's shuffle (random.shuffle) and swap (np.random in the
// worker processes) are unseeded; here both come from one seeded 64-bit generator, so a
// run is reproducible.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "common.h"
#include "image_io.h"

namespace oflow {
int launch_preprocess_pairs(const void* dev_raw, int npairs, int out_h, int out_w, float* out,
                            hipStream_t s);
}

using namespace oflow;

namespace {

constexpr size_t kAlign = 256;
inline size_t align_up(size_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

struct Slot {
  uint8_t* buf = nullptr;      // header (of_image_desc[2B]) + 2B image regions
  hipEvent_t copied = nullptr; // recorded after the H2D copy that last read this slot
  bool wait_copy = false;
  int64_t seq = -1;            // batch sequence number held / being decoded
  int remaining = 0;           // images still to decode (guarded by reader mutex)
  std::string err;
  std::vector<int32_t> pair, swapped;
};

struct Task {
  int slot, image;
  int64_t seq;
  std::string path;
};

}  // namespace

struct of_reader {
  std::vector<std::string> p1, p2;
  int batch = 0, nslots = 0, max_h = 0, max_w = 0;
  bool pinned = false;
  size_t header = 0, stride = 0, bytes = 0;
  std::mt19937_64 rng;
  std::vector<int> order;
  int nbatches = 0, next_batch_idx = 0;
  int64_t submitted = 0, consumed = 0;
  std::vector<Slot> slots;
  std::deque<Task> queue;
  std::mutex mu;
  std::condition_variable cv_task, cv_done;
  std::vector<std::thread> threads;
  bool stop = false;

  void shuffle() { std::shuffle(order.begin(), order.end(), rng); }

  // add_fetch_task (data_reader.py:110-119) for slot s; caller holds mu.
  void submit(int s) {
    Slot& sl = slots[s];
    sl.seq = submitted++;
    sl.err.clear();
    sl.remaining = 2 * batch;
    for (int i = 0; i < batch; ++i) {
      const int pi = order[(size_t)next_batch_idx * batch + i];
      const bool sw = (rng() >> 63) != 0;  // read_item: np.random.rand() < 0.5 keeps the order
      sl.pair[i] = pi;
      sl.swapped[i] = sw;
      queue.push_back({s, 2 * i, sl.seq, sw ? p2[pi] : p1[pi]});
      queue.push_back({s, 2 * i + 1, sl.seq, sw ? p1[pi] : p2[pi]});
    }
    if (next_batch_idx == nbatches - 1) {
      next_batch_idx = 0;
      shuffle();
    } else {
      ++next_batch_idx;
    }
    cv_task.notify_all();
  }

  void worker() {
    std::vector<uint8_t> file;
    for (;;) {
      Task t;
      bool wait_copy;
      hipEvent_t ev;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv_task.wait(lk, [&] { return stop || !queue.empty(); });
        if (stop) return;
        t = std::move(queue.front());
        queue.pop_front();
        wait_copy = slots[t.slot].wait_copy;
        ev = slots[t.slot].copied;
      }
      // the previous batch in this slot may still be in flight to the GPU
      std::string err;
      if (wait_copy && hipEventSynchronize(ev) != hipSuccess) err = "reader: hipEventSynchronize failed";
      Slot& sl = slots[t.slot];
      png::Info in;
      of_image_desc* descs = reinterpret_cast<of_image_desc*>(sl.buf);
      uint8_t* dst = sl.buf + header + (size_t)t.image * stride;
      if (err.empty() && png::read_file(t.path.c_str(), file, err)) {
        if (png::parse_info(file.data(), file.size(), in, err)) {
          if (in.h > max_h || in.w > max_w) {
            err = "reader: " + t.path + " is " + std::to_string(in.h) + "x" + std::to_string(in.w) +
                  ", larger than the reader's max " + std::to_string(max_h) + "x" +
                  std::to_string(max_w);
          } else if (png::decode_bgr(file.data(), file.size(), dst, stride, in, err)) {
            descs[t.image].offset = (int64_t)(header + (size_t)t.image * stride);
            descs[t.image].h = in.h;
            descs[t.image].w = in.w;
          } else {
            err += ": " + t.path;
          }
        }
      }
      std::lock_guard<std::mutex> lk(mu);
      if (!err.empty() && sl.err.empty()) sl.err = err;
      if (--sl.remaining == 0) cv_done.notify_all();
    }
  }

  // Wait for the next batch in submission order; returns its slot (caller holds lk).
  int wait_next(std::unique_lock<std::mutex>& lk) {
    const int s = (int)(consumed % nslots);
    cv_done.wait(lk, [&] { return slots[s].remaining == 0; });
    return s;
  }

  ~of_reader() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv_task.notify_all();
    for (auto& t : threads) t.join();
    for (auto& s : slots) {
      if (s.copied) {
        (void)hipEventSynchronize(s.copied);
        (void)hipEventDestroy(s.copied);
      }
      if (s.buf) {
        if (pinned) (void)hipHostFree(s.buf);
        else free(s.buf);
      }
    }
  }
};

extern "C" {

int of_png_scan(int n, const char* const* paths, int nthreads, int* max_h, int* max_w) {
  OF_CHECK_ARG(n >= 0 && (n == 0 || paths) && max_h && max_w, "png_scan: bad arguments");
  nthreads = std::max(1, std::min(nthreads, 64));
  std::atomic<int> next{0}, mh{0}, mw{0};
  std::mutex emu;
  std::string first_err;
  auto run = [&] {
    for (int i; (i = next++) < n;) {
      png::Info in;
      std::string err;
      if (!png::file_info(paths[i], in, err)) {
        std::lock_guard<std::mutex> lk(emu);
        if (first_err.empty()) first_err = err;
        continue;
      }
      for (int v = mh.load(); in.h > v && !mh.compare_exchange_weak(v, in.h);) {}
      for (int v = mw.load(); in.w > v && !mw.compare_exchange_weak(v, in.w);) {}
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nthreads; ++t) th.emplace_back(run);
  run();
  for (auto& t : th) t.join();
  if (!first_err.empty()) return fail(OF_EINVAL, "png_scan: " + first_err);
  *max_h = mh.load();
  *max_w = mw.load();
  return OF_OK;
}

int of_reader_create(int npairs, const char* const* path1, const char* const* path2, int batch,
                     int nworkers, int nslots, int max_h, int max_w, uint64_t seed, int pinned,
                     of_reader** out) {
  OF_CHECK_ARG(out && path1 && path2, "reader_create: null argument");
  OF_CHECK_ARG(batch > 0 && npairs >= batch, "reader_create: need at least one full batch "
               "(nbatches = npairs // batch_size, data_reader.py:86)");
  OF_CHECK_ARG(nworkers >= 1 && nworkers <= 256 && nslots >= 1 && nslots <= 64,
               "reader_create: nworkers in [1, 256], nslots in [1, 64]");
  OF_CHECK_ARG(max_h > 0 && max_w > 0 && (int64_t)max_h * max_w <= (1ll << 26),
               "reader_create: bad max image size");
  *out = nullptr;
  auto* r = new of_reader();
  r->batch = batch;
  r->nslots = nslots;
  r->max_h = max_h;
  r->max_w = max_w;
  r->pinned = pinned != 0;
  r->rng.seed(seed);
  for (int i = 0; i < npairs; ++i) {
    if (!path1[i] || !path2[i]) {
      delete r;
      return fail(OF_EINVAL, "reader_create: null path");
    }
    r->p1.emplace_back(path1[i]);
    r->p2.emplace_back(path2[i]);
  }
  r->order.resize(npairs);
  for (int i = 0; i < npairs; ++i) r->order[i] = i;
  r->nbatches = npairs / batch;
  r->header = align_up(sizeof(of_image_desc) * 2 * batch);
  r->stride = align_up((size_t)max_h * max_w * 3);
  r->bytes = r->header + r->stride * 2 * batch;
  r->slots.resize(nslots);
  for (auto& s : r->slots) {
    s.pair.resize(batch);
    s.swapped.resize(batch);
    if (r->pinned) {
      if (hipHostMalloc(reinterpret_cast<void**>(&s.buf), r->bytes, hipHostMallocDefault) != hipSuccess ||
          hipEventCreateWithFlags(&s.copied, hipEventDisableTiming) != hipSuccess) {
        s.buf = nullptr;
        delete r;
        return fail(OF_EHIP, "reader_create: pinned slot allocation failed");
      }
    } else {
      s.buf = static_cast<uint8_t*>(malloc(r->bytes));
      if (!s.buf) {
        delete r;
        return fail(OF_EINVAL, "reader_create: out of host memory");
      }
    }
    memset(s.buf, 0, r->bytes);
  }
  {
    std::lock_guard<std::mutex> lk(r->mu);
    r->shuffle();                                   // AsyncReader.__init__ (:91)
    for (int s = 0; s < nslots; ++s) r->submit(s);  // the first fetch tasks (:92-93)
  }
  for (int t = 0; t < nworkers; ++t) r->threads.emplace_back([r] { r->worker(); });
  *out = r;
  return OF_OK;
}

int64_t of_reader_raw_bytes(const of_reader* r) { return r ? (int64_t)r->bytes : -1; }

int of_reader_nbatches(const of_reader* r) { return r ? r->nbatches : -1; }

// Host variant of of_reader_next (no GPU): copies the next raw batch (descriptor header +
// BGR frames, the layout of_preprocess_pairs reads) into dst.
int of_reader_next_host(of_reader* r, void* dst, int64_t cap, int32_t* pair_index,
                        int32_t* swapped) {
  OF_CHECK_ARG(r && dst, "reader_next_host: null argument");
  OF_CHECK_ARG(cap >= (int64_t)r->bytes, "reader_next_host: destination smaller than "
               "of_reader_raw_bytes()");
  std::unique_lock<std::mutex> lk(r->mu);
  const int s = r->wait_next(lk);
  Slot& sl = r->slots[s];
  if (!sl.err.empty()) {
    const std::string e = sl.err;
    ++r->consumed;
    r->submit(s);
    return fail(OF_EINVAL, e);
  }
  memcpy(dst, sl.buf, r->bytes);
  if (pair_index) std::copy(sl.pair.begin(), sl.pair.end(), pair_index);
  if (swapped) std::copy(sl.swapped.begin(), sl.swapped.end(), swapped);
  ++r->consumed;
  sl.wait_copy = false;
  r->submit(s);
  return OF_OK;
}

int of_reader_next(of_reader* r, void* dev_raw, int64_t cap, float* out, int out_h, int out_w,
                   int32_t* pair_index, int32_t* swapped, void* stream) {
  OF_CHECK_ARG(r && dev_raw && out, "reader_next: null argument");
  OF_CHECK_ARG(r->pinned, "reader_next: the reader was created without pinned slots "
               "(use of_reader_next_host)");
  OF_CHECK_ARG(cap >= (int64_t)r->bytes, "reader_next: device buffer smaller than "
               "of_reader_raw_bytes()");
  OF_CHECK_ARG(out_h > 0 && out_w > 0, "reader_next: bad output size");
  hipStream_t st = as_stream(stream);
  std::unique_lock<std::mutex> lk(r->mu);
  const int s = r->wait_next(lk);
  Slot& sl = r->slots[s];
  if (!sl.err.empty()) {
    const std::string e = sl.err;
    ++r->consumed;
    sl.wait_copy = false;
    r->submit(s);
    return fail(OF_EINVAL, e);
  }
  if (hipMemcpyAsync(dev_raw, sl.buf, r->bytes, hipMemcpyHostToDevice, st) != hipSuccess)
    return fail(OF_EHIP, "reader_next: hipMemcpyAsync failed");
  int rc = launch_preprocess_pairs(dev_raw, r->batch, out_h, out_w, out, st);
  if (rc != OF_OK) return rc;
  if (hipEventRecord(sl.copied, st) != hipSuccess) return fail(OF_EHIP, "reader_next: hipEventRecord failed");
  if (pair_index) std::copy(sl.pair.begin(), sl.pair.end(), pair_index);
  if (swapped) std::copy(sl.swapped.begin(), sl.swapped.end(), swapped);
  sl.wait_copy = true;
  ++r->consumed;
  r->submit(s);
  return OF_OK;
}

int of_reader_destroy(of_reader* r) {
  delete r;
  return OF_OK;
}

}  // extern "C"
