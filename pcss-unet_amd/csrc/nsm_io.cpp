// Frame loader of the hot path's input side:
// the reference's `.npy` frame files ({split}_inputs.npy f32 [N,C,H,W],
// {split}_labels.npy f64/f32 [N,1,H,W], prepare_dataset.py:47,71-72) are
// memory-mapped; worker threads copy the frames of upcoming batches out of
// the page cache into pinned host slots (labels converted to f32 on the way,
// setdata.py:322); `nsm_loader_next` hands a ready slot to the caller's HIP
// stream as two async H2D copies and records an event that guards the slot's
// reuse. Normalisation ((x - mean_c) / (std_c + 1e-8), setdata.py:316) is a
// GPU kernel (nsm_normalize_frames), so the host threads only move bytes.
//
// The batch order is the reference's (DataLoader shuffle=False, main.py:850):
// this rank's contiguous shard [r*N/W, (r+1)*N/W), batches in order, the last
// one short; after the last batch the loader starts the next epoch.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "nsm_common.h"

namespace nsm {

struct Npy {
  int fd = -1;
  const unsigned char* map = nullptr;
  size_t map_len = 0, data_off = 0;
  int dtype = -1;  // 0 f32, 1 f64
  std::vector<int64_t> shape;
  size_t elem = 0;
};

// NPY v1/v2/v3 header: magic, version, header_len, python-dict literal
static bool parse_npy_header(const unsigned char* p, size_t len, Npy& a, std::string& err) {
  if (len < 10 || memcmp(p, "\x93NUMPY", 6) != 0) {
    err = "not an .npy file";
    return false;
  }
  const int major = p[6];
  size_t hlen, hoff;
  if (major == 1) {
    hlen = p[8] | (p[9] << 8);
    hoff = 10;
  } else if (major == 2 || major == 3) {
    if (len < 12) return err = "truncated header", false;
    hlen = (size_t)p[8] | ((size_t)p[9] << 8) | ((size_t)p[10] << 16) | ((size_t)p[11] << 24);
    hoff = 12;
  } else {
    err = "unsupported .npy version";
    return false;
  }
  if (hoff + hlen > len) return err = "truncated header", false;
  std::string h((const char*)p + hoff, hlen);
  auto field = [&](const char* key) -> std::string {
    size_t k = h.find(key);
    if (k == std::string::npos) return "";
    size_t c = h.find(':', k);
    return c == std::string::npos ? "" : h.substr(c + 1);
  };
  std::string d = field("'descr'");
  if (d.find("<f4") != std::string::npos || d.find("|f4") != std::string::npos) {
    a.dtype = 0;
    a.elem = 4;
  } else if (d.find("<f8") != std::string::npos) {
    a.dtype = 1;
    a.elem = 8;
  } else {
    err = "dtype must be little-endian float32 or float64";
    return false;
  }
  std::string f = field("'fortran_order'");
  if (f.find("True") != std::string::npos && f.find("True") < f.find(',')) {
    err = "fortran_order arrays are not supported";
    return false;
  }
  std::string s = field("'shape'");
  size_t lp = s.find('('), rp = s.find(')');
  if (lp == std::string::npos || rp == std::string::npos) return err = "bad shape", false;
  std::string dims = s.substr(lp + 1, rp - lp - 1);
  a.shape.clear();
  size_t i = 0;
  while (i < dims.size()) {
    while (i < dims.size() && (dims[i] == ' ' || dims[i] == ',')) ++i;
    if (i >= dims.size()) break;
    size_t j = i;
    while (j < dims.size() && dims[j] >= '0' && dims[j] <= '9') ++j;
    if (j == i) return err = "bad shape", false;
    a.shape.push_back(std::stoll(dims.substr(i, j - i)));
    i = j;
  }
  a.data_off = hoff + hlen;
  return true;
}

static bool open_npy(const char* path, Npy& a, std::string& err) {
  a.fd = open(path, O_RDONLY);
  if (a.fd < 0) return err = std::string("cannot open ") + path, false;
  struct stat st;
  if (fstat(a.fd, &st) != 0) return err = "fstat failed", false;
  a.map_len = (size_t)st.st_size;
  void* m = mmap(nullptr, a.map_len, PROT_READ, MAP_SHARED, a.fd, 0);
  if (m == MAP_FAILED) return err = "mmap failed", false;
  a.map = (const unsigned char*)m;
  if (!parse_npy_header(a.map, a.map_len, a, err)) return false;
  size_t n = a.elem;
  for (int64_t d : a.shape) n *= (size_t)d;
  if (a.data_off + n > a.map_len) return err = std::string(path) + ": file shorter than its shape", false;
  return true;
}

static void close_npy(Npy& a) {
  if (a.map) munmap((void*)a.map, a.map_len);
  if (a.fd >= 0) close(a.fd);
  a.map = nullptr;
  a.fd = -1;
}

struct Slot {
  float* x = nullptr;  // pinned [batch][C][H][W]
  float* y = nullptr;  // pinned [batch][1][H][W] (f32)
  hipEvent_t ev = nullptr;
  int frames = 0;
  long long batch_id = -1;
  bool ready = false, in_flight = false;
};

struct Loader {
  Npy xin, yin;
  int batch = 0;
  long long lo = 0, hi = 0;  // this rank's frame range
  size_t x_frame = 0, y_frame = 0;  // floats per frame
  long long nbatches = 0;
  std::vector<Slot> slots;
  std::vector<std::thread> workers;
  std::mutex mu;
  std::condition_variable cv_work, cv_ready;
  std::deque<int> todo;  // slots to fill
  long long next_fill = 0, next_take = 0;
  bool stop = false;
  std::string error;
};

static void fill_slot(Loader& L, Slot& s, long long batch_id) {
  const long long b = batch_id % L.nbatches;
  const long long f0 = L.lo + b * L.batch;
  const long long f1 = std::min(L.hi, f0 + L.batch);
  s.frames = (int)(f1 - f0);
  const unsigned char* xs = L.xin.map + L.xin.data_off + (size_t)f0 * L.x_frame * 4;
  memcpy(s.x, xs, (size_t)s.frames * L.x_frame * 4);
  const unsigned char* ys = L.yin.map + L.yin.data_off + (size_t)f0 * L.y_frame * L.yin.elem;
  const size_t ny = (size_t)s.frames * L.y_frame;
  if (L.yin.dtype == 0) {
    memcpy(s.y, ys, ny * 4);
  } else {
    const double* yd = (const double*)ys;
    for (size_t i = 0; i < ny; ++i) s.y[i] = (float)yd[i];  // labels f64 -> f32
  }
}

static void worker_main(Loader* L) {
  for (;;) {
    int si;
    long long bid;
    {
      std::unique_lock<std::mutex> lk(L->mu);
      L->cv_work.wait(lk, [&] { return L->stop || !L->todo.empty(); });
      if (L->stop) return;
      si = L->todo.front();
      L->todo.pop_front();
      bid = L->next_fill++;
    }
    Slot& s = L->slots[si];
    if (s.ev) (void)hipEventSynchronize(s.ev);  // previous H2D from this slot has finished
    fill_slot(*L, s, bid);
    {
      std::lock_guard<std::mutex> lk(L->mu);
      s.batch_id = bid;
      s.ready = true;
    }
    L->cv_ready.notify_all();
  }
}

}  // namespace nsm

using namespace nsm;

extern "C" int nsm_npy_info(const char* path, int64_t* shape, int max_dims, int* ndim, int* dtype,
                            int64_t* data_offset) {
  NSM_CHECK_ARG(path && shape && ndim && dtype, "npy_info: null pointer");
  Npy a;
  std::string err;
  bool ok = open_npy(path, a, err);
  if (ok) {
    *ndim = (int)a.shape.size();
    for (int i = 0; i < (int)a.shape.size() && i < max_dims; ++i) shape[i] = a.shape[i];
    *dtype = a.dtype;
    if (data_offset) *data_offset = (int64_t)a.data_off;
  }
  close_npy(a);
  if (!ok) return fail(NSM_E_ARG, "npy_info: %s", err.c_str());
  return 0;
}

extern "C" void* nsm_loader_create(const char* inputs_path, const char* labels_path, int batch,
                                   int rank, int world, int nslots, int nthreads) {
  if (!inputs_path || !labels_path || batch < 1 || world < 1 || rank < 0 || rank >= world) {
    fail(NSM_E_ARG, "loader_create: bad args");
    return nullptr;
  }
  Loader* L = new Loader();
  std::string err;
  if (!open_npy(inputs_path, L->xin, err) || !open_npy(labels_path, L->yin, err)) {
    close_npy(L->xin);
    close_npy(L->yin);
    delete L;
    fail(NSM_E_ARG, "loader_create: %s", err.c_str());
    return nullptr;
  }
  if (L->xin.dtype != 0 || L->xin.shape.size() != 4 || L->yin.shape.size() != 4 ||
      L->xin.shape[0] != L->yin.shape[0] || L->yin.shape[1] != 1 ||
      L->xin.shape[2] != L->yin.shape[2] || L->xin.shape[3] != L->yin.shape[3]) {
    close_npy(L->xin);
    close_npy(L->yin);
    delete L;
    fail(NSM_E_ARG, "loader_create: expected inputs f32 [N,C,H,W] and labels [N,1,H,W]");
    return nullptr;
  }
  const long long N = L->xin.shape[0];
  L->lo = N * rank / world;  // nsm_amd.data.shard_range
  L->hi = N * (rank + 1) / world;
  L->batch = batch;
  L->x_frame = (size_t)L->xin.shape[1] * L->xin.shape[2] * L->xin.shape[3];
  L->y_frame = (size_t)L->yin.shape[2] * L->yin.shape[3];
  L->nbatches = (L->hi - L->lo + batch - 1) / batch;
  if (L->nbatches < 1) {
    close_npy(L->xin);
    close_npy(L->yin);
    delete L;
    fail(NSM_E_ARG, "loader_create: empty shard");
    return nullptr;
  }
  if (nslots < 2) nslots = 2;
  if (nthreads < 1) nthreads = 1;
  L->slots.resize(nslots);
  for (auto& s : L->slots) {
    if (hipHostMalloc((void**)&s.x, (size_t)batch * L->x_frame * 4, hipHostMallocDefault) !=
            hipSuccess ||
        hipHostMalloc((void**)&s.y, (size_t)batch * L->y_frame * 4, hipHostMallocDefault) !=
            hipSuccess ||
        hipEventCreateWithFlags(&s.ev, hipEventDisableTiming) != hipSuccess) {
      fail(NSM_E_HIP, "loader_create: pinned allocation failed");
      for (auto& t : L->slots) {
        if (t.x) (void)hipHostFree(t.x);
        if (t.y) (void)hipHostFree(t.y);
        if (t.ev) (void)hipEventDestroy(t.ev);
      }
      close_npy(L->xin);
      close_npy(L->yin);
      delete L;
      return nullptr;
    }
  }
  for (int i = 0; i < nslots; ++i) L->todo.push_back(i);
  for (int t = 0; t < nthreads; ++t) L->workers.emplace_back(worker_main, L);
  L->cv_work.notify_all();
  return L;
}

extern "C" int64_t nsm_loader_batches(void* h) {
  return h ? ((Loader*)h)->nbatches : 0;
}

extern "C" int nsm_loader_frame_dims(void* h, int* C, int* H, int* W) {
  NSM_CHECK_ARG(h && C && H && W, "loader_frame_dims: bad args");
  Loader* L = (Loader*)h;
  *C = (int)L->xin.shape[1];
  *H = (int)L->xin.shape[2];
  *W = (int)L->xin.shape[3];
  return 0;
}

// Copies the next batch into dev_x [frames][C][H][W] / dev_y [frames][1][H][W]
// (f32, raw) asynchronously on `stream`; returns the frame count (>0) or -1.
extern "C" int nsm_loader_next(void* h, void* dev_x, void* dev_y, void* stream) {
  if (!h || !dev_x || !dev_y) return fail(NSM_E_ARG, "loader_next: bad args"), -1;
  Loader* L = (Loader*)h;
  hipStream_t s = as_stream(stream);
  int si = -1;
  {
    std::unique_lock<std::mutex> lk(L->mu);
    const long long want = L->next_take;
    L->cv_ready.wait(lk, [&] {
      for (size_t i = 0; i < L->slots.size(); ++i)
        if (L->slots[i].ready && L->slots[i].batch_id == want) return true;
      return false;
    });
    for (size_t i = 0; i < L->slots.size(); ++i)
      if (L->slots[i].ready && L->slots[i].batch_id == want) si = (int)i;
    L->next_take++;
  }
  Slot& sl = L->slots[si];
  const int n = sl.frames;
  hipError_t e1 = hipMemcpyAsync(dev_x, sl.x, (size_t)n * L->x_frame * 4, hipMemcpyHostToDevice, s);
  hipError_t e2 = hipMemcpyAsync(dev_y, sl.y, (size_t)n * L->y_frame * 4, hipMemcpyHostToDevice, s);
  hipError_t e3 = hipEventRecord(sl.ev, s);
  {
    std::lock_guard<std::mutex> lk(L->mu);
    sl.ready = false;
    L->todo.push_back(si);  // the worker waits for sl.ev before overwriting
  }
  L->cv_work.notify_one();
  if (e1 != hipSuccess || e2 != hipSuccess || e3 != hipSuccess)
    return fail(NSM_E_HIP, "loader_next: %s", hipGetErrorString(e1 ? e1 : e2 ? e2 : e3)), -1;
  return n;
}

extern "C" void nsm_loader_destroy(void* h) {
  if (!h) return;
  Loader* L = (Loader*)h;
  {
    std::lock_guard<std::mutex> lk(L->mu);
    L->stop = true;
  }
  L->cv_work.notify_all();
  for (auto& t : L->workers) t.join();
  for (auto& s : L->slots) {
    if (s.ev) {
      (void)hipEventSynchronize(s.ev);
      (void)hipEventDestroy(s.ev);
    }
    if (s.x) (void)hipHostFree(s.x);
    if (s.y) (void)hipHostFree(s.y);
  }
  close_npy(L->xin);
  close_npy(L->yin);
  delete L;
}
