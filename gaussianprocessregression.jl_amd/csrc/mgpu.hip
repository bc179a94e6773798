// mgpu.hip -- split-kernel block prediction sharded over the GPUs of one node, in ONE host
// process (src/split_predict.jl:5-53 is the single-CPU reference).
//
// The grid rows e of x_{e,q} = xe_e + xq_q are independent once the training factor U and the
// weights wt = K^{-1} y exist:
//   1. fit  -- GPR_MGPU_BROADCAST: device 0 fits (K, tile-DAG POTRF, wt) and RCCL broadcasts
//              U's upper triangle (~4 N^2 bytes instead of 8 N^2) plus wt over xGMI; the
//              receivers unpack it into their U and drop their cached block inverses (rebuilt
//              from the received factor).  The broadcast is STREAMED: U leaves in ~16 chunks of
//              tile rows, each packed and broadcast as soon as the running tile-DAG launch has
//              finalised its rows (a gate kernel polls the launch's progress counters; the
//              launch leaves 8 CUs free for the gates, packs and RCCL kernels), so only the last
//              chunk and wt trail the factorisation instead of the whole 4.3 GB (C5).
//              GPR_MGPU_REPLICATE: every device fits for itself (no N^2 exchange: the fit is
//              ~180 ms at ns = 32768 while the packed broadcast moves 4.3 GB).
//   2. rows -- device i takes gpr_shard_pieces(ne, ngpu, i, var_lo, var_hi): an even share of
//              the variance rows (an ns^2 triangular solve per test point) and of the mean-only
//              rows, as at most three contiguous pieces, all in one split_predict_pieces call
//              (the ns x nq C factor built once per device), into output buffers sized to
//              the device's rows (compact: pieces concatenated), not to the grid.
//   3. out  -- every device copies its rows of mu (ne x nq column-major, index e + q ne) and of
//              the variance diagonal (index e nq + q) straight into the caller's host arrays
//              (each GPU over its own PCIe link; no gather through one device).
// One host thread per device drives phases 1-3 (each with the device current) and issues its
// own ungrouped RCCL calls on its communicator (no ncclGroupStart/End: each rank posts every
// chunk's broadcast, in the same order, from its own thread).  RCCL is loaded with dlopen, so
// libgpr_hip.so has no link-time dependency on it and a host process that already carries a
// librccl.so.1 (torch) shares that one.
#include <dlfcn.h>

#include <algorithm>
#include <array>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "common.hpp"

namespace {

struct RcclApi {
  void* h = nullptr;
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*Broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t,
                            hipStream_t) = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

// the process's librccl if one is loaded already, else the system's
bool load_rccl(RcclApi* r, std::string* err) {
  if (r->h) return true;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
  if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) {
    *err = std::string("cannot load librccl.so.1: ") + dlerror();
    return false;
  }
  r->CommInitAll = (decltype(r->CommInitAll))dlsym(h, "ncclCommInitAll");
  r->CommDestroy = (decltype(r->CommDestroy))dlsym(h, "ncclCommDestroy");
  r->Broadcast = (decltype(r->Broadcast))dlsym(h, "ncclBroadcast");
  r->GetErrorString = (decltype(r->GetErrorString))dlsym(h, "ncclGetErrorString");
  if (!r->CommInitAll || !r->CommDestroy || !r->Broadcast || !r->GetErrorString) {
    *err = "librccl.so.1 lacks an ncclCommInitAll / ncclCommDestroy / ncclBroadcast symbol";
    return false;
  }
  r->h = h;
  return true;
}

constexpr int PACK_NB = 128;

// packed upper triangle by 128-column blocks: block b = columns [128 b, j1) keeps rows [0, j1)
// of each of its columns, j1 = min(128 (b + 1), n); every block before the last is full, so
// block b starts at 128^2 b (b + 1) / 2
__host__ __device__ inline size_t pack_base(int b) {
  return (size_t)PACK_NB * PACK_NB * (size_t)b * (size_t)(b + 1) / 2;
}

size_t packed_len(int n) {
  const int nb = (n + PACK_NB - 1) / PACK_NB;
  return nb ? pack_base(nb - 1) + (size_t)(n - (nb - 1) * PACK_NB) * n : 0;
}

// one workgroup row-strip per column c: rows [0, j1) of column c <-> packed, coalesced both ways
template <bool PACK>
__global__ __launch_bounds__(256) void pack_upper_kernel(double* __restrict__ U, size_t ldu, int n,
                                                         double* __restrict__ P) {
  const int c = blockIdx.x;
  const int b = c / PACK_NB;
  const int j1 = min((b + 1) * PACK_NB, n);
  double* p = P + pack_base(b) + (size_t)(c - b * PACK_NB) * j1;
  double* u = U + (size_t)c * ldu;
  for (int r = blockIdx.y * 256 + threadIdx.x; r < j1; r += gridDim.y * 256) {
    if (PACK)
      p[r] = u[r];
    else
      u[r] = p[r];
  }
}

int launch_pack(gpr_ctx* ctx, double* U, int ldu, int n, double* P, bool pack) {
  if (n <= 0) return 0;
  const dim3 grid(n, std::min(32, (n + 255) / 256));
  if (pack)
    pack_upper_kernel<true><<<grid, 256, 0, ctx->stream>>>(U, (size_t)ldu, n, P);
  else
    pack_upper_kernel<false><<<grid, 256, 0, ctx->stream>>>(U, (size_t)ldu, n, P);
  LAUNCH_CHECK(ctx);
  return 0;
}

// ---- the streamed broadcast's layout: U's upper triangle by TILE ROWS ----------------------
// Tile row i (rows [128 i, 128 i + m_i), m_i = min(128, n - 128 i), columns [128 i, n)) as an
// m_i x (n - 128 i) column-major block, tile rows in order: the same elements as the
// column-block packing, ordered so that a prefix of tile rows is a prefix of the buffer.  The
// tile-DAG finalises U top-down by tile rows (left-looking, tickets by row), so a chunk of tile
// rows can leave for the other GPUs while the factorisation is still running below it.
__host__ __device__ inline size_t rows_base(int i, int n) {
  return (size_t)PACK_NB * ((size_t)i * n - (size_t)PACK_NB * i * (i - 1) / 2);
}

// tile rows [r0, r1) of U <-> their slice of the row layout (PACK: U -> P).  Workgroup x = column
// c of [128 r0, n): its rows [128 r0, min(128 r1, end of c's tile column)) are contiguous in U.
template <bool PACK>
__global__ __launch_bounds__(256) void rows_pack_kernel(double* __restrict__ U, size_t ldu, int n,
                                                        int r0, int r1, double* __restrict__ P) {
  const int c = PACK_NB * r0 + blockIdx.x;
  const int rend = min(min(PACK_NB * r1, n), PACK_NB * (c / PACK_NB + 1));
  for (int r = PACK_NB * r0 + blockIdx.y * 256 + threadIdx.x; r < rend; r += gridDim.y * 256) {
    const int i = r / PACK_NB;
    const int m = min(PACK_NB, n - PACK_NB * i);
    double* p = P + rows_base(i, n) + (size_t)(c - PACK_NB * i) * m + (r - PACK_NB * i);
    double* u = U + r + (size_t)c * ldu;
    if (PACK)
      *p = *u;
    else
      *u = *p;
  }
}

// Waits until tile rows [r0, r1) of U are final in a running tile-DAG launch: colprog[j] (final
// tiles at the top of tile column j, raised with sc1 stores after the tiles' sc1 stores drained)
// >= min(r1, j + 1) for every j >= r0, and ustored[j] for the diagonal tiles j in [r0, r1) (a
// diagonal task publishes colprog once W_j is out and stores U_jj after that).  Bounded like
// the DAG's own waits: after `limit` polls it flags *err and returns (the chunk then carries
// garbage and the host reports the error).
__global__ __launch_bounds__(256) void rows_gate_kernel(const int* __restrict__ colprog,
                                                        const int* __restrict__ ustored, int nt,
                                                        int r0, int r1, long long limit,
                                                        int* __restrict__ err) {
  long long spins = 0;
  for (;;) {
    int ok = limit > 0;  // (limit 0: give up at once)
    for (int j = r0 + (int)threadIdx.x; j < nt; j += 256)
      ok &= __hip_atomic_load(colprog + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >=
                min(r1, j + 1) &&
            (j >= r1 ||
             __hip_atomic_load(ustored + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0);
    if (__syncthreads_and(ok)) break;
    if (++spins > limit) {  // (spins is the same in every thread: a uniform exit)
      if (threadIdx.x == 0) atomicExch(err, 1);
      break;
    }
    __builtin_amdgcn_s_sleep(8);
  }
}

void launch_rows_pack(hipStream_t s, double* U, int ldu, int n, int r0, int r1, double* P,
                      bool pack) {
  const int rows = std::min(PACK_NB * r1, n) - PACK_NB * r0;
  const dim3 grid(n - PACK_NB * r0, std::min(8, (rows + 255) / 256));
  if (pack)
    rows_pack_kernel<true><<<grid, 256, 0, s>>>(U, (size_t)ldu, n, r0, r1, P);
  else
    rows_pack_kernel<false><<<grid, 256, 0, s>>>(U, (size_t)ldu, n, r0, r1, P);
}

// chunk boundaries in tile rows: about equal bytes per chunk, at most `maxc` chunks
std::vector<int> row_chunks(int n, int maxc) {
  const int nt = (n + PACK_NB - 1) / PACK_NB;
  const size_t total = packed_len(n);
  const int C = std::max(1, std::min(maxc, nt));
  std::vector<int> b{0};
  for (int i = 1; i < nt; ++i)
    if (rows_base(i, n) * C >= total * b.size() && (int)b.size() < C) b.push_back(i);
  b.push_back(nt);
  return b;
}

void shard_rows(int n, int world, int rank, int* lo, int* hi) {
  const int q = n / world, r = n % world;
  *lo = rank * q + std::min(rank, r);
  *hi = *lo + q + (rank < r ? 1 : 0);
}

}  // namespace

struct gpr_mgpu {
  int ngpu = 0;
  std::vector<int> dev;
  std::vector<gpr_ctx_t> ctx;
  std::vector<ncclComm_t> comm;
  RcclApi rccl;
  std::string err;
  struct Bufs {  // device buffers of one GPU, grown on demand
    double *x = nullptr, *y = nullptr, *xe = nullptr, *xq = nullptr, *U = nullptr, *wt = nullptr,
           *mu = nullptr, *var = nullptr, *pk = nullptr, *U2 = nullptr;
    size_t cx = 0, cy = 0, cxe = 0, cxq = 0, cU = 0, cwt = 0, cmu = 0, cvar = 0, cpk = 0, cU2 = 0;
  };
  std::vector<Bufs> buf;
  // device 0's stream for the streamed broadcast (gates, packs, RCCL), created after the
  // context's five: a stream whose hardware queue is shared with the factorisation's stream
  // (GPU_MAX_HW_QUEUES = 4) runs its work behind the launch, so everything goes on this one
  hipStream_t sp = nullptr;
  int* derr = nullptr;  // device 0: a gate timed out
  // knobs (kMgpuKnobs below): read from the environment once at gpr_mgpu_create, changed
  // with gpr_mgpu_set_knob (include/gpr_hip.h)
  int stream_out = -1;   // GPR_MGPU_STREAM: U streamed out during device 0's fit (-1: only at ngpu 1)
  int reserve_cu = 8;    // GPR_MGPU_RESERVE_CU: CUs the streamed fit's launch leaves free
  int chunks = 16;       // GPR_MGPU_CHUNKS: tile-row chunks of the broadcast
  int self_bcast = 0;    // (test build only) ngpu 1 runs the broadcast protocol to itself
};

namespace {

struct MgpuKnob {
  const char* name;
  int gpr_mgpu::*ip;
};
const MgpuKnob kMgpuKnobs[] = {
    {"GPR_MGPU_STREAM", &gpr_mgpu::stream_out},
    {"GPR_MGPU_RESERVE_CU", &gpr_mgpu::reserve_cu},
    {"GPR_MGPU_CHUNKS", &gpr_mgpu::chunks},
#ifdef GPR_TESTING
    // device 0 as its own receiver, so the one-GPU test box runs the broadcast protocol
    {"GPR_MGPU_SELF_BCAST", &gpr_mgpu::self_bcast},
#endif
};

void mgpu_knob_set(gpr_mgpu* h, const MgpuKnob& k, int v) {
  if (k.ip == &gpr_mgpu::stream_out) v = v < 0 ? -1 : (v != 0);
  if (k.ip == &gpr_mgpu::reserve_cu) v = std::max(0, v);
  if (k.ip == &gpr_mgpu::chunks) v = std::max(1, v);
  h->*k.ip = v;
}

const MgpuKnob* mgpu_knob_find(const char* name) {
  if (!name) return nullptr;
  for (const MgpuKnob& k : kMgpuKnobs)
    if (!strcmp(k.name, name)) return &k;
  return nullptr;
}

int mg_err(gpr_mgpu* h, int code, const char* fmt, ...) {
  char b[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(b, sizeof b, fmt, ap);
  va_end(ap);
  h->err = b;
  return code;
}

// (called with the device current)
bool grow(double** p, size_t* cap, size_t n) {
  if (*cap >= n && *p) return true;
  if (*p) hipFree(*p);
  *p = nullptr;
  *cap = 0;
  if (hipMalloc((void**)p, std::max<size_t>(n, 1) * sizeof(double)) != hipSuccess) return false;
  *cap = n;
  return true;
}

// elements of chunk [r0, r1) of tile rows in the row layout
size_t chunk_len(int r0, int r1, int n) {
  const int m = std::min(PACK_NB, n - PACK_NB * (r1 - 1));  // rows of the last tile row
  return rows_base(r1 - 1, n) - rows_base(r0, n) + (size_t)m * (n - PACK_NB * (r1 - 1));
}

// Device 0's side of the broadcast: chunk c = tile rows [rows[c], rows[c+1]) of U, packed into
// its slice of pk (behind a gate on the DAG's progress counters when streamed), then broadcast
// from that slice, all on stream sp (measured with one stream per role, pack and RCCL: the
// second stream shared the launch's hardware queue and its work ran after the launch).  Called
// from the tile-DAG launch's hook (streamed: the chunks run beside the factorisation, on the
// CUs its grid leaves free) or after the fit.
struct StreamOut {
  gpr_mgpu* h = nullptr;
  int n = 0;
  double *U = nullptr, *pk = nullptr, *U2 = nullptr;  // U2: self-broadcast receive buffer
  std::vector<int> rows;
  long long limit = 1ll << 27;  // gate polls (~minutes: a gate waits up to a whole fit)
  bool fired = false;  // chunks enqueued by the hook, beside the DAG launch
  int rc = 0;
  // fault injection (tests, GPR_MGPU_FAIL_UNPACK=k): every receiver's unpack of chunk k fails
  // (skipped, error recorded, protocol continued) -- the self-broadcast receiver included
  int fail_unpack = -1;
  int recv_rc = 0;  // the self-broadcast receiver's error (device 0 reports it at the end)
};

// (dep: the event the chunks wait for -- the counters' reset, or the end of the fit; null when
// the caller has already synchronised with the fit)
int enqueue_chunks(StreamOut* so, const int* colprog, const int* ustored, int nt, hipEvent_t dep) {
  gpr_mgpu* h = so->h;
  auto& R = h->rccl;
  // every chunk's broadcast is issued whatever fails on the way -- a failed launch, a failed
  // RCCL call -- because the receivers are already waiting in the matching calls; the first
  // error is returned after the last chunk and the host reports it
  int rc = 0;
  if (dep && hipStreamWaitEvent(h->sp, dep, 0) != hipSuccess) rc = GPR_E_HIP;
  for (size_t c = 0; c + 1 < so->rows.size(); ++c) {
    const int r0 = so->rows[c], r1 = so->rows[c + 1];
    double* slice = so->pk + rows_base(r0, so->n);
    const size_t len = chunk_len(r0, r1, so->n);
    if (colprog)
      rows_gate_kernel<<<1, 256, 0, h->sp>>>(colprog, ustored, nt, r0, r1, so->limit, h->derr);
    launch_rows_pack(h->sp, so->U, so->n, so->n, r0, r1, so->pk, true);
    if (hipGetLastError() != hipSuccess && !rc) rc = GPR_E_HIP;
    if (R.Broadcast(slice, slice, len, ncclDouble, 0, h->comm[0], h->sp) != ncclSuccess && !rc)
      rc = GPR_E_HIP;
    if (so->U2 && !so->recv_rc) {  // the self-broadcast receiver's unpack
      if ((int)c == so->fail_unpack)
        so->recv_rc = GPR_E_HIP;
      else
        launch_rows_pack(h->sp, so->U2, so->n, so->n, r0, r1, so->pk, false);
      if (hipGetLastError() != hipSuccess) so->recv_rc = GPR_E_HIP;
    }
  }
  return rc;
}

// The tile-DAG launch's hook on device 0 (called right after the launch is enqueued): the
// gates, packs and broadcasts go on sp behind the counters' reset, i.e. beside the launch.
// A padded copy (other shapes) or a missing event: nothing here, the chunks follow the fit.
void stream_out_hook(void* user, const double* dA, int n, int lda, const int* colprog,
                     const int* ustored, int nt, hipEvent_t counters_reset) {
  auto* so = static_cast<StreamOut*>(user);
  if (!counters_reset || !ustored || dA != so->U || n != so->n || lda != so->n) return;
  so->rc = enqueue_chunks(so, colprog, ustored, nt, counters_reset);
  so->fired = true;
  // the gates poll the launch's counters (ctx->dag_sync) on sp: the context's next DAG launch
  // waits for them before it resets or reallocates that buffer
  gpr_ctx* c = so->h->ctx[0];
  if (!c->dag_sync_readers &&
      hipEventCreateWithFlags(&c->dag_sync_readers, hipEventDisableTiming) != hipSuccess)
    c->dag_sync_readers = nullptr;
  if (c->dag_sync_readers && hipEventRecord(c->dag_sync_readers, so->h->sp) == hipSuccess)
    c->dag_sync_readers_pending = true;
  else if (hipStreamSynchronize(so->h->sp) != hipSuccess && !so->rc)  // (no event: drain now)
    so->rc = GPR_E_HIP;
  (void)hipGetLastError();
}

// run f(i) for every device on its own host thread (device i current), collect return codes
template <class F>
std::vector<int> on_devices(gpr_mgpu* h, F f) {
  std::vector<int> rc(h->ngpu, 0);
  std::vector<std::thread> th;
  for (int i = 0; i < h->ngpu; ++i)
    th.emplace_back([&, i] {
      if (hipSetDevice(h->dev[i]) != hipSuccess) {
        rc[i] = GPR_E_HIP;
        return;
      }
      rc[i] = f(i);
    });
  for (auto& t : th) t.join();
  return rc;
}

}  // namespace

extern "C" {

int gpr_shard_pieces(int n, int world, int rank, int v_lo, int v_hi, int* pieces) {
  if (n < 0 || world <= 0 || rank < 0 || rank >= world || !pieces) return GPR_E_ARG;
  v_lo = std::max(0, std::min(v_lo, n));
  v_hi = std::max(0, std::min(v_hi, n));
  const int nv = std::max(v_hi - v_lo, 0);
  int raw[6], np = 0, a, b;
  if (nv) {
    shard_rows(nv, world, rank, &a, &b);
    if (b > a) {
      raw[2 * np] = v_lo + a;
      raw[2 * np + 1] = v_lo + b;
      ++np;
    }
  }
  shard_rows(n - nv, world, rank, &a, &b);  // mean-only index i < v_lo is row i, else i + nv
  if (a < std::min(b, v_lo)) {
    raw[2 * np] = a;
    raw[2 * np + 1] = std::min(b, v_lo);
    ++np;
  }
  const int lo2 = std::max(a, v_lo), hi2 = b;
  if (hi2 > lo2) {
    raw[2 * np] = lo2 + nv;
    raw[2 * np + 1] = hi2 + nv;
    ++np;
  }
  // sort by start, merge adjacent pieces
  for (int i = 1; i < np; ++i)
    for (int j = i; j > 0 && raw[2 * j] < raw[2 * (j - 1)]; --j) {
      std::swap(raw[2 * j], raw[2 * (j - 1)]);
      std::swap(raw[2 * j + 1], raw[2 * (j - 1) + 1]);
    }
  int m = 0;
  for (int i = 0; i < np; ++i) {
    if (m && pieces[2 * m - 1] == raw[2 * i]) {
      pieces[2 * m - 1] = raw[2 * i + 1];
    } else {
      pieces[2 * m] = raw[2 * i];
      pieces[2 * m + 1] = raw[2 * i + 1];
      ++m;
    }
  }
  return m;
}

int gpr_pack_upper(gpr_ctx_t ctx, const double* dU, int n, int ldu, double* dP) {
  if (n < 0 || ldu < std::max(n, 1) || (n && (!dU || !dP))) return set_err(ctx, GPR_E_ARG, "bad args");
  return launch_pack(ctx, const_cast<double*>(dU), ldu, n, dP, true);
}

int gpr_unpack_upper(gpr_ctx_t ctx, const double* dP, int n, double* dU, int ldu) {
  if (n < 0 || ldu < std::max(n, 1) || (n && (!dU || !dP))) return set_err(ctx, GPR_E_ARG, "bad args");
  return launch_pack(ctx, dU, ldu, n, const_cast<double*>(dP), false);
}

size_t gpr_packed_upper_len(int n) { return n > 0 ? packed_len(n) : 0; }

int gpr_mgpu_create(int ngpu, const int* devices, gpr_mgpu_t* out) {
  if (!out || ngpu <= 0 || !devices) return GPR_E_ARG;
  *out = nullptr;
  gpr_mgpu* h = new gpr_mgpu();
  h->ngpu = ngpu;
  h->dev.assign(devices, devices + ngpu);
  h->ctx.assign(ngpu, nullptr);
  h->buf.resize(ngpu);
  // the handle's documented knobs (include/gpr_hip.h), read once here; gpr_mgpu_set_knob
  // changes them on a live handle
  for (const MgpuKnob& k : kMgpuKnobs)
    if (const char* e = getenv(k.name)) mgpu_knob_set(h, k, atoi(e));
  for (int i = 0; i < ngpu; ++i) {
    for (int j = 0; j < i; ++j)
      if (h->dev[j] == h->dev[i]) {
        gpr_mgpu_destroy(h);
        return GPR_E_ARG;  // one rank per GPU (RCCL refuses two on one device)
      }
    if (gpr_ctx_create(h->dev[i], nullptr, &h->ctx[i]) != 0) {
      gpr_mgpu_destroy(h);
      return GPR_E_HIP;
    }
  }
  if (hipSetDevice(h->dev[0]) != hipSuccess || hipMalloc((void**)&h->derr, sizeof(int)) != hipSuccess) {
    gpr_mgpu_destroy(h);
    return GPR_E_HIP;
  }
  {
    // low priority.  Measured (profiles/r03_mgpu_stream_out_trace.txt): low, normal and high
    // priority streams all ran the stream-out inside the launch's window; a CU-masked stream
    // ran it after the launch.
    int lo = 0, hi = 0;
    hipDeviceGetStreamPriorityRange(&lo, &hi);
    const hipError_t r = hipStreamCreateWithPriority(&h->sp, hipStreamNonBlocking, lo);
    if (r != hipSuccess) {
      h->sp = nullptr;
      gpr_mgpu_destroy(h);
      return GPR_E_HIP;
    }
  }
  std::string err;
  if (!load_rccl(&h->rccl, &err)) {
    gpr_mgpu_destroy(h);
    return GPR_E_UNSUP;
  }
  h->comm.assign(ngpu, nullptr);
  if (h->rccl.CommInitAll(h->comm.data(), ngpu, h->dev.data()) != ncclSuccess) {
    h->comm.clear();
    gpr_mgpu_destroy(h);
    return GPR_E_HIP;
  }
  *out = h;
  return 0;
}

int gpr_mgpu_destroy(gpr_mgpu_t h) {
  if (!h) return 0;
  for (int i = 0; i < h->ngpu; ++i) {
    if (hipSetDevice(h->dev[i]) != hipSuccess) continue;
    if (i < (int)h->comm.size() && h->comm[i] && h->rccl.CommDestroy) h->rccl.CommDestroy(h->comm[i]);
    auto& b = h->buf[i];
    for (double* p : {b.x, b.y, b.xe, b.xq, b.U, b.wt, b.mu, b.var, b.pk, b.U2})
      if (p) hipFree(p);
    if (i == 0) {
      if (h->sp) hipStreamDestroy(h->sp);
      if (h->derr) hipFree(h->derr);
    }
    if (h->ctx[i]) gpr_ctx_destroy(h->ctx[i]);
  }
  delete h;
  return 0;
}

const char* gpr_mgpu_last_error(gpr_mgpu_t h) { return h ? h->err.c_str() : "null handle"; }

int gpr_mgpu_set_knob(gpr_mgpu_t h, const char* name, double value) {
  if (!h) return GPR_E_ARG;
  const MgpuKnob* k = mgpu_knob_find(name);
  if (!k) return mg_err(h, GPR_E_ARG, "unknown knob %s", name ? name : "(null)");
  mgpu_knob_set(h, *k, (int)value);
  return 0;
}

int gpr_mgpu_get_knob(gpr_mgpu_t h, const char* name, double* value) {
  if (!h || !value) return GPR_E_ARG;
  const MgpuKnob* k = mgpu_knob_find(name);
  if (!k) return mg_err(h, GPR_E_ARG, "unknown knob %s", name ? name : "(null)");
  *value = (double)(h->*k->ip);
  return 0;
}

int gpr_split_predict_mgpu(gpr_mgpu_t h, const int* kinds, int nk, const double* hp, int d,
                           const double* X, int ns, const double* y, const double* Xe, int ne,
                           const double* Xq, int nq, int var_lo, int var_hi, double eps,
                           int fit_mode, double* mu, double* var, int* info) {
  if (!h) return GPR_E_ARG;
  if (info) *info = 0;
  if (ns <= 0 || ne <= 0 || nq <= 0 || d <= 0 || !X || !y || !Xe || !Xq || !mu || !var || !kinds ||
      !hp)
    return mg_err(h, GPR_E_ARG, "bad args");
  if (fit_mode != GPR_MGPU_BROADCAST && fit_mode != GPR_MGPU_REPLICATE)
    return mg_err(h, GPR_E_ARG, "fit_mode %d is neither GPR_MGPU_BROADCAST nor _REPLICATE", fit_mode);
  const int G = h->ngpu;
  // GPR_MGPU_SELF_BCAST=1 (tests on a one-GPU box): the broadcast path even for one device,
  // which then also acts as a receiver (pack, 1-rank RCCL broadcast, unpack, forget)
  const bool self_bcast = h->self_bcast != 0;
  const bool bcast = fit_mode == GPR_MGPU_BROADCAST && (G > 1 || self_bcast);
  const size_t npk = packed_len(ns);
  std::vector<int> finfo(G, 0);
  // each device's row pieces (its output buffers hold just these rows)
  std::vector<std::array<int, 6>> pcs(G);
  std::vector<int> npc(G), rows(G, 0);
  for (int i = 0; i < G; ++i) {
    npc[i] = gpr_shard_pieces(ne, G, i, var_lo, var_hi, pcs[i].data());
    if (npc[i] < 0) return mg_err(h, GPR_E_ARG, "bad shard");
    for (int k = 0; k < npc[i]; ++k) rows[i] += pcs[i][2 * k + 1] - pcs[i][2 * k];
  }
  // Broadcast protocol (every device runs it in full, whatever happens to the fit, so no
  // receiver is left waiting in RCCL): chunks of tile rows of U in the row layout (about equal
  // bytes, at most GPR_MGPU_CHUNKS = 16), then wt.  Streamed: device 0's factorisation leaves
  // GPR_MGPU_RESERVE_CU (8) CUs free and each chunk is packed and broadcast beside it as soon as
  // its tile rows are final; the receivers unpack each chunk as it lands, and only the last
  // chunk and wt trail the factorisation.  GPR_MGPU_STREAM default: streamed on one device (the
  // self-broadcast path the tests run), after the fit across devices -- no run with two or more
  // GPUs has exercised the streamed receivers yet; GPR_MGPU_STREAM=1 opts in there.
  const bool stream = h->stream_out >= 0 ? h->stream_out != 0 : G == 1;
  const int reserve = std::max(0, h->reserve_cu);
  const int maxc = std::max(1, h->chunks);
  StreamOut so;
  so.h = h;
  so.n = ns;
  so.rows = row_chunks(ns, maxc);
  // (tests: GPR_MGPU_GATE_LIMIT=0 makes every gate give up at once -- the error path whatever
  // the factorisation's progress)
#ifdef GPR_TESTING
  // fault injection, test builds only (libgpr_hip_testing.so; tests/fault_scenarios.py)
  if (const char* e = getenv("GPR_MGPU_GATE_LIMIT")) so.limit = std::max(0ll, atoll(e));
  if (const char* e = getenv("GPR_MGPU_FAIL_UNPACK")) so.fail_unpack = atoi(e);
#endif
  // 0. buffers and inputs on every device (a failure here stops every device before the
  //    broadcast protocol starts)
  auto rc = on_devices(h, [&](int i) -> int {
    gpr_ctx_t c = h->ctx[i];
    auto& b = h->buf[i];
    if (!grow(&b.x, &b.cx, (size_t)d * ns) || !grow(&b.y, &b.cy, ns) ||
        !grow(&b.xe, &b.cxe, (size_t)d * ne) || !grow(&b.xq, &b.cxq, (size_t)d * nq) ||
        !grow(&b.U, &b.cU, (size_t)ns * ns) || !grow(&b.wt, &b.cwt, ns) ||
        !grow(&b.mu, &b.cmu, (size_t)std::max(rows[i], 1) * nq) ||
        !grow(&b.var, &b.cvar, (size_t)std::max(rows[i], 1) * nq) ||
        (bcast && !grow(&b.pk, &b.cpk, npk)) ||
        (bcast && self_bcast && !grow(&b.U2, &b.cU2, (size_t)ns * ns)))
      return set_err(c, GPR_E_NOMEM, "device %d: allocation failed", h->dev[i]);
    GPR_TRY(gpr_upload(c, b.x, X, sizeof(double) * d * ns));
    GPR_TRY(gpr_upload(c, b.y, y, sizeof(double) * ns));
    GPR_TRY(gpr_upload(c, b.xe, Xe, sizeof(double) * d * ne));
    GPR_TRY(gpr_upload(c, b.xq, Xq, sizeof(double) * d * nq));
    if (i == 0) HIP_TRY(c, hipMemset(h->derr, 0, sizeof(int)));
    return gpr_sync(c);
  });
  for (int i = 0; i < G; ++i)
    if (rc[i] != 0)
      return mg_err(h, rc[i] < 0 ? rc[i] : GPR_E_HIP, "device %d: %s", h->dev[i],
                    gpr_last_error(h->ctx[i]));
  // 1. device 0 (or every device) fits; device 0 sends U and wt, the receivers take them
  rc = on_devices(h, [&](int i) -> int {
    gpr_ctx_t c = h->ctx[i];
    auto& b = h->buf[i];
    if (!bcast) {
      const int r = gpr_fit(c, kinds, nk, hp, d, b.x, ns, b.y, 1, ns, eps, b.U, ns, b.wt, &finfo[i]);
      if (r != 0) return r;  // (> 0: the LAPACK info)
      return gpr_sync(c);
    }
    auto& R = h->rccl;
    hipStream_t s = (hipStream_t)gpr_ctx_stream(c);
    if (i > 0) {  // receiver: every chunk, unpacked as it lands, then wt
      // every broadcast is posted whatever fails (device 0 sends them all): after an error
      // the remaining chunks are still received -- not unpacked -- and the error is reported
      // once the protocol is complete, so neither side is left waiting in RCCL
      int err = 0;
      std::string what;
      for (size_t k = 0; k + 1 < so.rows.size(); ++k) {
        const int r0 = so.rows[k], r1 = so.rows[k + 1];
        double* slice = b.pk + rows_base(r0, ns);
        const size_t len = chunk_len(r0, r1, ns);
        if (R.Broadcast(slice, slice, len, ncclDouble, 0, h->comm[i], s) != ncclSuccess) {
          if (!err) err = GPR_E_HIP, what = "RCCL broadcast of chunk " + std::to_string(k);
          continue;
        }
        if (err) continue;
        if ((int)k == so.fail_unpack) {
          err = GPR_E_HIP;
          what = "unpack of chunk " + std::to_string(k) + " (injected fault)";
          continue;
        }
        launch_rows_pack(s, b.U, ns, ns, r0, r1, b.pk, false);
        if (hipGetLastError() != hipSuccess)
          err = GPR_E_HIP, what = "unpack of chunk " + std::to_string(k);
      }
      if (R.Broadcast(b.wt, b.wt, ns, ncclDouble, 0, h->comm[i], s) != ncclSuccess && !err)
        err = GPR_E_HIP, what = "RCCL broadcast of wt";
      const int src = gpr_sync(c);
      if (err) return set_err(c, err, "receiver: %s failed", what.c_str());
      if (src) return src;
      return gpr_forget_factor(c);  // the inverses of this buffer's old contents are stale
    }
    // device 0: fit with the hook armed, then whatever the hook did not send, then wt
    so.U = b.U;
    so.pk = b.pk;
    so.U2 = self_bcast ? b.U2 : nullptr;
    if (stream) {
      c->dag_hook = stream_out_hook;
      c->dag_hook_user = &so;
      c->dag_reserve_cu = reserve;
    }
    const int r = gpr_fit(c, kinds, nk, hp, d, b.x, ns, b.y, 1, ns, eps, b.U, ns, b.wt, &finfo[0]);
    c->dag_hook = nullptr;
    c->dag_reserve_cu = 0;
    (void)hipGetLastError();  // (a failed fit must not stop the protocol below)
    int prc = so.fired ? so.rc : 0;
    // wt (and, unless streamed, U) leave after the fit: behind an event, or -- if none can be
    // made -- after a host sync; the protocol runs to its end whatever failed
    hipEvent_t fit_done = nullptr;
    if (hipEventCreateWithFlags(&fit_done, hipEventDisableTiming) != hipSuccess) fit_done = nullptr;
    if (fit_done && hipEventRecord(fit_done, s) != hipSuccess) {
      hipEventDestroy(fit_done);
      fit_done = nullptr;
    }
    if (!fit_done && hipStreamSynchronize(s) != hipSuccess && !prc) prc = GPR_E_HIP;
    (void)hipGetLastError();
    if (!so.fired) {
      const int r2 = enqueue_chunks(&so, nullptr, nullptr, 0, fit_done);
      if (!prc) prc = r2;
    }
    if (fit_done && hipStreamWaitEvent(h->sp, fit_done, 0) != hipSuccess && !prc) prc = GPR_E_HIP;
    if (R.Broadcast(b.wt, b.wt, ns, ncclDouble, 0, h->comm[0], h->sp) != ncclSuccess && !prc)
      prc = GPR_E_HIP;
    if (fit_done) hipEventDestroy(fit_done);
    if (hipStreamSynchronize(h->sp) != hipSuccess && !prc) prc = GPR_E_HIP;
    c->dag_sync_readers_pending = false;  // (sp drained: the gates are done)
    if (r != 0) return r;
    if (prc != 0) return set_err(c, GPR_E_HIP, "device 0: streaming U / wt out failed");
    int herr = 0;
    HIP_TRY(c, hipMemcpy(&herr, h->derr, sizeof(int), hipMemcpyDeviceToHost));
    if (herr) return set_err(c, GPR_E_HIP, "device 0: a tile-row gate timed out");
    if (so.recv_rc)
      return set_err(c, so.recv_rc, "device 0 (self-broadcast receiver): unpack of chunk %d failed%s",
                     so.fail_unpack, so.fail_unpack >= 0 ? " (injected fault)" : "");
    if (self_bcast) GPR_TRY(gpr_forget_factor(c));
    return gpr_sync(c);
  });
  for (int i = 0; i < G; ++i) {
    if (finfo[i] > 0) {
      if (info) *info = finfo[i];
      return mg_err(h, finfo[i], "device %d: K is not positive definite (info %d)", h->dev[i],
                    finfo[i]);
    }
    if (rc[i] < 0)
      return mg_err(h, rc[i], "device %d: %s", h->dev[i], gpr_last_error(h->ctx[i]));
  }
  // 2. every device predicts its rows and copies them into the host arrays
  rc = on_devices(h, [&](int i) -> int {
    gpr_ctx_t c = h->ctx[i];
    auto& b = h->buf[i];
    const double* U = (bcast && self_bcast) ? b.U2 : b.U;  // (self: the received copy)
    const int* pieces = pcs[i].data();
    const int np = npc[i], R = std::max(rows[i], 1);
    // the shard's rows only (compact: piece k's rows at off_k, mu leading dimension R)
    GPR_TRY(split_predict_pieces(c, kinds, nk, hp, d, b.x, ns, U, ns, b.wt, b.xe, ne, b.xq, nq,
                                 pieces, np, var_lo, var_hi, eps, b.mu, R, b.var, true));
    hipStream_t s = (hipStream_t)gpr_ctx_stream(c);
    for (int k = 0, off = 0; k < np; off += pieces[2 * k + 1] - pieces[2 * k], ++k) {
      const int lo = pieces[2 * k], hi = pieces[2 * k + 1];
      HIP_TRY(c, hipMemcpy2DAsync(mu + lo, sizeof(double) * ne, b.mu + off, sizeof(double) * R,
                                  sizeof(double) * (hi - lo), nq, hipMemcpyDeviceToHost, s));
      HIP_TRY(c, hipMemcpyAsync(var + (size_t)lo * nq, b.var + (size_t)off * nq,
                                sizeof(double) * (size_t)(hi - lo) * nq, hipMemcpyDeviceToHost, s));
    }
    return gpr_sync(c);
  });
  for (int i = 0; i < G; ++i)
    if (rc[i] != 0)
      return mg_err(h, rc[i] < 0 ? rc[i] : GPR_E_HIP, "device %d: %s", h->dev[i],
                    gpr_last_error(h->ctx[i]));
  return 0;
}

}  // extern "C"
