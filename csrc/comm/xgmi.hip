// Direct-peer collectives over xGMI for tensor/sequence-parallel messages.
//
// An MI355X node is a fully connected graph: every GPU has 7 point-to-point xGMI links.  A ring
// collective (RCCL's default for these sizes) moves every byte over ONE link per direction per
// step; a direct-peer collective has each GPU read its 7 peers concurrently, i.e. over 7
// distinct links at once.  That is the pattern here:
//
//   * Every rank owns one symmetric workspace: [data: capacity bytes][signals: 2 x 64 x u32],
//     allocated uncached (hipDeviceMallocUncached) and exported with hipIpcGetMemHandle; every
//     rank maps all peers' workspaces (hipIpcOpenMemHandle), so a kernel can load or store
//     peer HBM directly.
//   * A collective = stage -> barrier -> pull -> barrier, four launches on the caller's stream:
//       stage   copy the input into the own workspace (many workgroups, 16-byte vectors)
//       barrier one wave: store `epoch` into slot [me] of every peer's signal row (system-scope
//               release), then spin until all peers' stores arrived in the own row (acquire);
//               the spin is bounded in wall time (s_memrealtime): a missing peer sets an
//               error word and the wave exits, so a broken peer can never hang the GPU
//       pull    all_gather: out[r] = peer_r.data[0:shard];  reduce_scatter: out = sum_r
//               peer_r.data[me*shard : (me+1)*shard] (f32 accumulation);  all_reduce:
//               out = sum_r peer_r.data (one-shot).  Workgroups are dealt round-robin over
//               the peers (workgroup b reads peer (b + me) % world first), so all links
//               carry traffic at once.
//       barrier the "done" row: nobody restages its workspace while a peer may still read it.
//     Kernel boundaries give the acquire/release of the data itself (caches are written back
//     at the end of a kernel and invalidated at the start of the next).
//   * Epochs increase monotonically per communicator, so signal rows never need resetting.
//   * A timed-out barrier is sticky: the error word stays set and every later barrier kernel of
//     the communicator returns at once, so one missing peer costs one timeout, not one per
//     collective; the trainer polls it (`check()`) and exits non-zero.
//   * Zero-copy: every collective takes the byte `offset` of its message in the workspace.  When
//     the input already lives there (a producer GEMM wrote its output straight into
//     `workspace()`, parallel/async_tp.py), the stage copy is skipped; peers pull from the same
//     offset of their own workspace.
//   * Copy-engine variants (`*_dma`): the stage and every peer pull are hipMemcpyAsync transfers
//     issued on a pool of per-peer streams forked from / joined into the caller's stream with
//     events, so the world-1 peer copies run concurrently on the copy engines (one xGMI link
//     each) and take no CU time; the reduce-scatter's sum is one local kernel over the pulled
//     slices.
//
// RCCL stays the path for the large DDP/ZeRO/FSDP buckets and for inter-node traffic.
// All stores are vector-memory stores / atomics; nothing writes through the scalar cache.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

namespace dtg {
namespace xgmi {

constexpr int kMaxRanks = 8;
constexpr int kSigSlots = 64;  // u32 per signal row (rank slots; padded to a 256-B row)

#define XGMI_CHECK(expr)                                                                         \
  do {                                                                                           \
    hipError_t _e = (expr);                                                                      \
    TORCH_CHECK(_e == hipSuccess, "xgmi: ", #expr, " failed: ", hipGetErrorString(_e));          \
  } while (0)

struct Peers {
  uint8_t* data[kMaxRanks];
  uint32_t* sig[kMaxRanks];
};

// ------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------
__global__ void barrier_kernel(Peers peers, int me, int world, int row, uint32_t epoch, uint32_t* err,
                               uint64_t timeout_ticks) {
  const int t = threadIdx.x;
  // a previous collective of this communicator timed out: peers are out of step, never wait again
  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) return;
  if (t < world) {
    uint32_t* dst = peers.sig[t] + row * kSigSlots + me;
    __hip_atomic_store(dst, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  if (t < world) {
    const uint32_t* src = peers.sig[me] + row * kSigSlots + t;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (true) {
      const uint32_t v = __hip_atomic_load(src, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      if ((int32_t)(v - epoch) >= 0) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
        __hip_atomic_store(err, 1u + (uint32_t)t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// dst[i] = src[i] for n16 16-byte vectors.
__global__ void copy16_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst, int64_t n16) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

// out[r * shard + i] = peer_r.data[i]; workgroups split as (peer, slice).
__global__ void all_gather_kernel(Peers peers, int me, int world, u32x4* __restrict__ out, int64_t shard16,
                                  int blocks_per_peer) {
  const int p = (blockIdx.x / blocks_per_peer + me) % world;
  const int b = blockIdx.x % blocks_per_peer;
  const u32x4* src = reinterpret_cast<const u32x4*>(peers.data[p]);
  u32x4* dst = out + (int64_t)p * shard16;
  for (int64_t i = (int64_t)b * blockDim.x + threadIdx.x; i < shard16; i += (int64_t)blocks_per_peer * blockDim.x)
    dst[i] = __builtin_nontemporal_load(src + i);
}

__device__ __forceinline__ void acc8_bf16(float* a, u32x4 v) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    a[2 * j] += __uint_as_float(v[j] << 16);
    a[2 * j + 1] += __uint_as_float(v[j] & 0xffff0000u);
  }
}

__device__ __forceinline__ u32x4 pack8_bf16(const float* a) {
  u32x4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t lo = __builtin_bit_cast(uint16_t, static_cast<__bf16>(a[2 * j]));
    const uint32_t hi = __builtin_bit_cast(uint16_t, static_cast<__bf16>(a[2 * j + 1]));
    r[j] = lo | (hi << 16);
  }
  return r;
}

// out[i] = sum_r peer_r.data[offset16 + i] over n16 vectors; IS_BF16 selects 8 x bf16 or 4 x f32
// per 16-byte vector.  Each workgroup reads its slice from every peer, starting at a different
// peer per workgroup so the links are loaded evenly.
template <bool IS_BF16>
__global__ void reduce_kernel(Peers peers, int me, int world, u32x4* __restrict__ out, int64_t offset16, int64_t n16) {
  const int first = (blockIdx.x + me) % world;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x) {
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < world; ++k) {
      const int p = (first + k) % world;
      const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(peers.data[p]) + offset16 + i);
      if constexpr (IS_BF16) {
        acc8_bf16(a, v);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] += __uint_as_float(v[j]);
      }
    }
    if constexpr (IS_BF16) {
      out[i] = pack8_bf16(a);
    } else {
      u32x4 r;
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = __float_as_uint(a[j]);
      out[i] = r;
    }
  }
}

// ------------------------------------------------------------------------------------------
// communicator
// ------------------------------------------------------------------------------------------
struct Comm {
  int rank = 0, world = 1, device = 0;
  int64_t capacity = 0;  // data bytes per rank
  uint8_t* base = nullptr;  // own workspace: data + signals
  uint32_t* err = nullptr;  // host-pinned error word
  Peers peers{};
  std::vector<void*> opened;
  uint32_t epoch = 0;
  double timeout_s = 60.0;
  // shared buffers (alloc_shared): every rank's copy of a buffer with the same layout, mapped
  // from every peer; shared[slot][r] = rank r's base (own or IPC-mapped)
  std::vector<std::vector<uint8_t*>> shared;
  std::vector<void*> shared_opened;
  // copy-engine path: one stream per peer, fork/join events
  hipStream_t peer_st[kMaxRanks] = {};
  hipEvent_t ev_fork = nullptr;
  hipEvent_t ev_join[kMaxRanks] = {};

  void ensure_streams() {
    if (ev_fork) return;
    for (int r = 0; r < world; ++r) {
      XGMI_CHECK(hipStreamCreateWithFlags(&peer_st[r], hipStreamNonBlocking));
      XGMI_CHECK(hipEventCreateWithFlags(&ev_join[r], hipEventDisableTiming));
    }
    XGMI_CHECK(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
  }

  ~Comm() {
    if (ev_fork) {
      (void)hipDeviceSynchronize();
      for (int r = 0; r < world; ++r) {
        (void)hipStreamDestroy(peer_st[r]);
        (void)hipEventDestroy(ev_join[r]);
      }
      (void)hipEventDestroy(ev_fork);
    }
    for (void* p : opened) (void)hipIpcCloseMemHandle(p);
    for (void* p : shared_opened) (void)hipIpcCloseMemHandle(p);
    if (base) (void)hipFree(base);
    if (err) (void)hipHostFree(err);
  }
  uint32_t* sig_of(uint8_t* b) const { return reinterpret_cast<uint32_t*>(b + capacity); }
};

std::mutex g_mu;
std::vector<std::unique_ptr<Comm>> g_comms;

Comm& get(int64_t id) {
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(id >= 0 && id < (int64_t)g_comms.size() && g_comms[id], "xgmi: bad communicator id ", id);
  return *g_comms[id];
}

int64_t create(int64_t capacity, int64_t rank, int64_t world, int64_t device) {
  TORCH_CHECK(world >= 1 && world <= kMaxRanks, "xgmi: world size must be 1..", kMaxRanks);
  TORCH_CHECK(rank >= 0 && rank < world, "xgmi: bad rank");
  TORCH_CHECK(capacity > 0 && capacity % 4096 == 0, "xgmi: capacity must be a positive multiple of 4096");
  auto c = std::make_unique<Comm>();
  c->rank = rank;
  c->world = world;
  c->device = device;
  c->capacity = capacity;
  c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, device));
  const size_t bytes = capacity + 2 * kSigSlots * sizeof(uint32_t);
  XGMI_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&c->base), bytes, hipDeviceMallocUncached));
  XGMI_CHECK(hipMemset(c->base + capacity, 0, 2 * kSigSlots * sizeof(uint32_t)));
  XGMI_CHECK(hipHostMalloc(reinterpret_cast<void**>(&c->err), sizeof(uint32_t), hipHostMallocCoherent));
  *c->err = 0;
  XGMI_CHECK(hipDeviceSynchronize());
  std::lock_guard<std::mutex> lk(g_mu);
  g_comms.push_back(std::move(c));
  return (int64_t)g_comms.size() - 1;
}

at::Tensor ipc_handle(int64_t id) {
  Comm& c = get(id);
  c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, c.device));
  hipIpcMemHandle_t h;
  XGMI_CHECK(hipIpcGetMemHandle(&h, c.base));
  auto t = at::empty({(int64_t)sizeof(h)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(t.data_ptr(), &h, sizeof(h));
  return t;
}

void open_peers(int64_t id, const at::Tensor& handles) {
  Comm& c = get(id);
  TORCH_CHECK(handles.device().is_cpu() && handles.scalar_type() == at::kByte && handles.dim() == 2 &&
                  handles.size(0) == c.world && handles.size(1) == (int64_t)sizeof(hipIpcMemHandle_t),
              "xgmi: handles must be a CPU uint8 tensor [world, ", sizeof(hipIpcMemHandle_t), "]");
  auto hc = handles.contiguous();
  c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, c.device));
  for (int r = 0; r < c.world; ++r) {
    uint8_t* p = nullptr;
    if (r == c.rank) {
      p = c.base;
    } else {
      hipIpcMemHandle_t h;
      std::memcpy(&h, hc.data_ptr<uint8_t>() + r * sizeof(h), sizeof(h));
      void* q = nullptr;
      XGMI_CHECK(hipIpcOpenMemHandle(&q, h, hipIpcMemLazyEnablePeerAccess));
      c.opened.push_back(q);
      p = static_cast<uint8_t*>(q);
    }
    c.peers.data[r] = p;
    c.peers.sig[r] = c.sig_of(p);
  }
}

void set_timeout(int64_t id, double seconds) { get(id).timeout_s = seconds; }

int64_t error(int64_t id) {
  Comm& c = get(id);
  return (int64_t)__atomic_load_n(c.err, __ATOMIC_ACQUIRE);
}

void destroy(int64_t id) {
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(id >= 0 && id < (int64_t)g_comms.size(), "xgmi: bad id");
  g_comms[id].reset();
}

at::Tensor workspace(int64_t id) {
  Comm& c = get(id);
  // a view of the own data region (no deleter: the communicator owns the memory)
  return at::from_blob(c.base, {c.capacity},
                       at::TensorOptions().dtype(at::kByte).device(c10::Device(c10::DeviceType::CUDA, c.device)));
}

// A fresh tensor (its own TensorImpl and version counter, not a view) over `sizes` elements of
// `dtype` at byte `offset` of the own data region: a zero-copy producer output.  Autograd forbids
// in-place changes to the base of a view a custom Function returned, and every hand-out of a
// slot rewrites the same memory, so each hand-out must be a distinct base.
at::Tensor workspace_view(int64_t id, int64_t offset, at::IntArrayRef sizes, at::ScalarType dtype) {
  Comm& c = get(id);
  int64_t n = 1;
  for (auto v : sizes) n *= v;
  const int64_t bytes = n * (int64_t)c10::elementSize(dtype);
  TORCH_CHECK(offset >= 0 && offset % 16 == 0 && offset + bytes <= c.capacity, "xgmi: workspace_view out of range");
  return at::from_blob(c.base + offset, sizes,
                       at::TensorOptions().dtype(dtype).device(c10::Device(c10::DeviceType::CUDA, c.device)));
}

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void barrier(Comm& c, int row, hipStream_t st) {
  // s_memrealtime runs at 100 MHz on gfx950.
  const uint64_t ticks = (uint64_t)(c.timeout_s * 1e8);
  barrier_kernel<<<1, 64, 0, st>>>(c.peers, c.rank, c.world, row, c.epoch, c.err, ticks);
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

int grid_for(int64_t n16, int cap = 2048) {
  int64_t g = (n16 + 255) / 256;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}

void check_io(const Comm& c, const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.get_device() == c.device, "xgmi: ", what, " must be on cuda:", c.device);
  TORCH_CHECK(t.is_contiguous(), "xgmi: ", what, " must be contiguous");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kFloat, "xgmi: ", what, " must be bf16 or f32");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0 && (t.numel() * t.element_size()) % 16 == 0,
              "xgmi: ", what, " must be 16-byte aligned and a multiple of 16 bytes");
}

void check_msg(const Comm& c, int64_t offset, int64_t bytes) {
  TORCH_CHECK(offset >= 0 && offset % 16 == 0, "xgmi: workspace offset must be a non-negative multiple of 16");
  TORCH_CHECK(offset + bytes <= c.capacity, "xgmi: message of ", bytes, " B at offset ", offset,
              " exceeds the workspace (", c.capacity, " B)");
}

// The output must not alias the message in the workspace: peers are still pulling from it while
// this rank writes its result.
void check_no_alias(const Comm& c, const at::Tensor& out, int64_t offset, int64_t bytes) {
  const auto lo = reinterpret_cast<uintptr_t>(out.data_ptr());
  const auto hi = lo + out.numel() * out.element_size();
  const auto wlo = reinterpret_cast<uintptr_t>(c.base + offset);
  TORCH_CHECK(hi <= wlo || lo >= wlo + bytes, "xgmi: the output overlaps the message in the workspace");
}

// The message's home in the own workspace; the stage copy is skipped when the producer already
// wrote it there (zero-copy).
uint8_t* stage(Comm& c, const at::Tensor& inp, int64_t offset, bool dma, hipStream_t st) {
  uint8_t* dst = c.base + offset;
  if (inp.data_ptr() == dst) return dst;
  const int64_t bytes = inp.numel() * inp.element_size();
  if (dma) {
    XGMI_CHECK(hipMemcpyAsync(dst, inp.data_ptr(), bytes, hipMemcpyDeviceToDevice, st));
  } else {
    const int64_t n16 = bytes / 16;
    copy16_kernel<<<grid_for(n16), 256, 0, st>>>(reinterpret_cast<const u32x4*>(inp.data_ptr()),
                                                 reinterpret_cast<u32x4*>(dst), n16);
    C10_HIP_KERNEL_LAUNCH_CHECK();
  }
  return dst;
}

// Copy-engine fan-out: the peer streams start after everything queued on `st` ...
void fork(Comm& c, hipStream_t st) {
  c.ensure_streams();
  XGMI_CHECK(hipEventRecord(c.ev_fork, st));
  for (int r = 0; r < c.world; ++r) XGMI_CHECK(hipStreamWaitEvent(c.peer_st[r], c.ev_fork, 0));
}

// ... and `st` continues once every peer copy has landed.
void join(Comm& c, hipStream_t st) {
  for (int r = 0; r < c.world; ++r) {
    XGMI_CHECK(hipEventRecord(c.ev_join[r], c.peer_st[r]));
    XGMI_CHECK(hipStreamWaitEvent(st, c.ev_join[r], 0));
  }
}

}  // namespace

void all_gather(int64_t id, const at::Tensor& out, const at::Tensor& inp, int64_t offset) {
  Comm& c = get(id);
  check_io(c, inp, "input");
  check_io(c, out, "output");
  TORCH_CHECK(out.scalar_type() == inp.scalar_type() && out.numel() == inp.numel() * c.world, "xgmi all_gather: shape");
  const int64_t bytes = inp.numel() * inp.element_size();
  check_msg(c, offset, bytes);
  check_no_alias(c, out, offset, bytes);
  c10::DeviceGuard g(inp.device());
  hipStream_t st = cur_stream();
  ++c.epoch;
  stage(c, inp, offset, false, st);
  barrier(c, 0, st);
  Peers src = c.peers;
  for (int r = 0; r < c.world; ++r) src.data[r] += offset;
  const int64_t shard16 = bytes / 16;
  const int bpp = std::max(1, grid_for(shard16, 1024));
  all_gather_kernel<<<bpp * c.world, 256, 0, st>>>(src, c.rank, c.world, reinterpret_cast<u32x4*>(out.data_ptr()),
                                                   shard16, bpp);
  C10_HIP_KERNEL_LAUNCH_CHECK();
  barrier(c, 1, st);
}

// Copy-engine all-gather: stage -> barrier -> world concurrent pulls (one per peer stream) ->
// barrier.  Only the two one-wave barrier kernels touch the shader array, so an all-gather on a
// side stream overlaps GEMMs without taking CUs from them (parallel/async_tp.py).
void all_gather_dma(int64_t id, const at::Tensor& out, const at::Tensor& inp, int64_t offset) {
  Comm& c = get(id);
  check_io(c, inp, "input");
  check_io(c, out, "output");
  TORCH_CHECK(out.scalar_type() == inp.scalar_type() && out.numel() == inp.numel() * c.world, "xgmi all_gather: shape");
  const int64_t bytes = inp.numel() * inp.element_size();
  check_msg(c, offset, bytes);
  check_no_alias(c, out, offset, bytes);
  c10::DeviceGuard g(inp.device());
  hipStream_t st = cur_stream();
  ++c.epoch;
  stage(c, inp, offset, true, st);
  barrier(c, 0, st);
  auto* o = static_cast<uint8_t*>(out.data_ptr());
  fork(c, st);
  for (int k = 0; k < c.world; ++k) {
    const int p = (c.rank + k) % c.world;
    const uint8_t* src = p == c.rank ? static_cast<const uint8_t*>(inp.data_ptr()) : c.peers.data[p] + offset;
    XGMI_CHECK(hipMemcpyAsync(o + (int64_t)p * bytes, src, bytes, hipMemcpyDeviceToDevice, c.peer_st[p]));
  }
  join(c, st);
  barrier(c, 1, st);
}

void reduce_scatter(int64_t id, const at::Tensor& out, const at::Tensor& inp, int64_t offset) {
  Comm& c = get(id);
  check_io(c, inp, "input");
  check_io(c, out, "output");
  TORCH_CHECK(out.scalar_type() == inp.scalar_type() && inp.numel() == out.numel() * c.world, "xgmi reduce_scatter: shape");
  const int64_t bytes = inp.numel() * inp.element_size();
  check_msg(c, offset, bytes);
  check_no_alias(c, out, offset, bytes);
  c10::DeviceGuard g(inp.device());
  hipStream_t st = cur_stream();
  ++c.epoch;
  stage(c, inp, offset, false, st);
  barrier(c, 0, st);
  const int64_t n16 = out.numel() * out.element_size() / 16;
  auto* o = reinterpret_cast<u32x4*>(out.data_ptr());
  Peers src = c.peers;
  for (int r = 0; r < c.world; ++r) src.data[r] += offset;
  if (inp.scalar_type() == at::kBFloat16)
    reduce_kernel<true><<<grid_for(n16), 256, 0, st>>>(src, c.rank, c.world, o, (int64_t)c.rank * n16, n16);
  else
    reduce_kernel<false><<<grid_for(n16), 256, 0, st>>>(src, c.rank, c.world, o, (int64_t)c.rank * n16, n16);
  C10_HIP_KERNEL_LAUNCH_CHECK();
  barrier(c, 1, st);
}

// Copy-engine reduce-scatter: the world slices [me*shard, (me+1)*shard) of every peer's message
// are pulled concurrently into a local [world, shard] scratch (one copy per peer stream), the
// peers are released, and one local kernel sums the slices at HBM speed (f32 accumulation).
void reduce_scatter_dma(int64_t id, const at::Tensor& out, const at::Tensor& inp, int64_t offset) {
  Comm& c = get(id);
  check_io(c, inp, "input");
  check_io(c, out, "output");
  TORCH_CHECK(out.scalar_type() == inp.scalar_type() && inp.numel() == out.numel() * c.world, "xgmi reduce_scatter: shape");
  const int64_t bytes = inp.numel() * inp.element_size();
  const int64_t shard = bytes / c.world;
  check_msg(c, offset, bytes);
  check_no_alias(c, out, offset, bytes);
  c10::DeviceGuard g(inp.device());
  hipStream_t st = cur_stream();
  // allocated on `st`; every peer-stream access is joined back into `st` before it is freed
  at::Tensor scratch = at::empty({bytes}, inp.options().dtype(at::kByte));
  auto* sc = static_cast<uint8_t*>(scratch.data_ptr());
  ++c.epoch;
  stage(c, inp, offset, true, st);
  barrier(c, 0, st);
  fork(c, st);
  for (int k = 0; k < c.world; ++k) {
    const int p = (c.rank + k) % c.world;
    const uint8_t* src = (p == c.rank ? static_cast<const uint8_t*>(inp.data_ptr()) : c.peers.data[p] + offset) +
                         (int64_t)c.rank * shard;
    XGMI_CHECK(hipMemcpyAsync(sc + (int64_t)p * shard, src, shard, hipMemcpyDeviceToDevice, c.peer_st[p]));
  }
  join(c, st);
  barrier(c, 1, st);  // peers may restage: the slices are local now
  Peers loc{};
  for (int r = 0; r < c.world; ++r) loc.data[r] = sc + (int64_t)r * shard;
  const int64_t n16 = shard / 16;
  auto* o = reinterpret_cast<u32x4*>(out.data_ptr());
  if (inp.scalar_type() == at::kBFloat16)
    reduce_kernel<true><<<grid_for(n16), 256, 0, st>>>(loc, c.rank, c.world, o, 0, n16);
  else
    reduce_kernel<false><<<grid_for(n16), 256, 0, st>>>(loc, c.rank, c.world, o, 0, n16);
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

void all_reduce(int64_t id, const at::Tensor& inout, int64_t offset) {
  Comm& c = get(id);
  check_io(c, inout, "tensor");
  const int64_t bytes = inout.numel() * inout.element_size();
  check_msg(c, offset, bytes);
  // in place: the result overwrites `inout`, so it must live outside the workspace message
  check_no_alias(c, inout, offset, bytes);
  c10::DeviceGuard g(inout.device());
  hipStream_t st = cur_stream();
  ++c.epoch;
  stage(c, inout, offset, false, st);
  barrier(c, 0, st);
  const int64_t n16 = bytes / 16;
  auto* o = reinterpret_cast<u32x4*>(inout.data_ptr());
  Peers src = c.peers;
  for (int r = 0; r < c.world; ++r) src.data[r] += offset;
  if (inout.scalar_type() == at::kBFloat16)
    reduce_kernel<true><<<grid_for(n16), 256, 0, st>>>(src, c.rank, c.world, o, 0, n16);
  else
    reduce_kernel<false><<<grid_for(n16), 256, 0, st>>>(src, c.rank, c.world, o, 0, n16);
  C10_HIP_KERNEL_LAUNCH_CHECK();
  barrier(c, 1, st);
}

// ------------------------------------------------------------------------------------------
// Shared buffers: data-parallel bucket collectives without staging (parallel/xgmi_dp.py)
// ------------------------------------------------------------------------------------------
// A buffer every rank allocates with the same size and layout (ZeRO's flat parameter and
// gradient buffers), IPC-exported and mapped from every peer.  Collectives on it are copy-engine
// pulls at arbitrary byte ranges of the peers' copies: a reduce-scatter pulls this rank's slice
// of a bucket from every peer into a local scratch and sums it; an all-gather pulls every peer's
// updated slice straight into place.  Only the one-wave barrier kernel and the local reduce
// touch the shader array.  Memory is ordinary (cached, coarse-grained) device memory, unlike the
// uncached workspace above, because no kernel here reads a peer's copy while that peer may still
// be writing it.  The workspace is read by pull KERNELS that poll peer flags mid-kernel, which
// needs fine-grained (uncached) memory.  Here every cross-device access is a copy-engine
// transfer, and each one is separated from the kernels that produce or consume the data by
// kernel boundaries.  Coarse-grained memory is coherent at those boundaries:
//  * producer side: the kernel that wrote a bucket ends with a release that writes its dirty L2
//    lines back to HBM, and only then does the barrier kernel after it on the stream signal the
//    peers whose copy engines read the bucket;
//  * consumer side: copy-engine writes go to HBM, not into this GPU's L2, and the next kernel that
//    reads the destination starts with an acquire that invalidates the L2's stale lines.
// (All xGMI tests so far share one GPU, so this is the HIP coarse-grained rule, not yet a
// cross-device measurement; the bench's N > 1 xGMI child checks replica checksums on a real node.)

// Own allocation; the tensor's deleter frees it (peers keep their mapping until they close it).
at::Tensor alloc_shared(int64_t id, int64_t nbytes) {
  Comm& c = get(id);
  TORCH_CHECK(nbytes > 0, "xgmi: alloc_shared needs a positive size");
  c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, c.device));
  void* p = nullptr;
  XGMI_CHECK(hipMalloc(&p, (size_t)nbytes));
  XGMI_CHECK(hipMemset(p, 0, (size_t)nbytes));
  XGMI_CHECK(hipDeviceSynchronize());
  {
    std::lock_guard<std::mutex> lk(g_mu);
    c.shared.push_back(std::vector<uint8_t*>(c.world, nullptr));
    c.shared.back()[c.rank] = static_cast<uint8_t*>(p);
  }
  const int dev = c.device;
  return at::from_blob(p, {nbytes}, [dev](void* q) {
           c10::DeviceGuard gg(c10::Device(c10::DeviceType::CUDA, dev));
           (void)hipFree(q);
         },
         at::TensorOptions().dtype(at::kByte).device(c10::Device(c10::DeviceType::CUDA, c.device)));
}

at::Tensor shared_handle(int64_t id, int64_t slot) {
  Comm& c = get(id);
  TORCH_CHECK(slot >= 0 && slot < (int64_t)c.shared.size(), "xgmi: bad shared slot");
  c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, c.device));
  hipIpcMemHandle_t h;
  XGMI_CHECK(hipIpcGetMemHandle(&h, c.shared[slot][c.rank]));
  auto t = at::empty({(int64_t)sizeof(h)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(t.data_ptr(), &h, sizeof(h));
  return t;
}

void open_shared(int64_t id, int64_t slot, const at::Tensor& handles) {
  Comm& c = get(id);
  TORCH_CHECK(slot >= 0 && slot < (int64_t)c.shared.size(), "xgmi: bad shared slot");
  TORCH_CHECK(handles.device().is_cpu() && handles.scalar_type() == at::kByte && handles.dim() == 2 &&
                  handles.size(0) == c.world && handles.size(1) == (int64_t)sizeof(hipIpcMemHandle_t),
              "xgmi: handles must be a CPU uint8 tensor [world, ", sizeof(hipIpcMemHandle_t), "]");
  auto hc = handles.contiguous();
  c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, c.device));
  for (int r = 0; r < c.world; ++r) {
    if (r == c.rank) continue;
    hipIpcMemHandle_t h;
    std::memcpy(&h, hc.data_ptr<uint8_t>() + r * sizeof(h), sizeof(h));
    void* q = nullptr;
    XGMI_CHECK(hipIpcOpenMemHandle(&q, h, hipIpcMemLazyEnablePeerAccess));
    c.shared_opened.push_back(q);
    c.shared[slot][r] = static_cast<uint8_t*>(q);
  }
}

// Everyone's work queued before this point on their stream has finished (signal + wait, bounded).
void signal_wait(int64_t id) {
  Comm& c = get(id);
  c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, c.device));
  ++c.epoch;
  barrier(c, 0, cur_stream());
}

// dst[dst_off[p] : + nbytes[p]] = peer p's shared slot [src_off[p] : + nbytes[p]] for every peer
// p != this rank, one hipMemcpyAsync per peer on that peer's stream (the copy engines, all
// links at once), forked from and joined back into the caller's stream.  Offsets / sizes: CPU
// int64 [world].
void pull(int64_t id, int64_t slot, const at::Tensor& dst, const at::Tensor& src_off, const at::Tensor& nbytes,
          const at::Tensor& dst_off) {
  Comm& c = get(id);
  TORCH_CHECK(slot >= 0 && slot < (int64_t)c.shared.size(), "xgmi: bad shared slot");
  TORCH_CHECK(dst.is_cuda() && dst.get_device() == c.device && dst.is_contiguous(), "xgmi pull: dst");
  for (const at::Tensor* t : {&src_off, &nbytes, &dst_off})
    TORCH_CHECK(t->device().is_cpu() && t->scalar_type() == at::kLong && t->numel() == c.world,
                "xgmi pull: offsets / sizes must be CPU int64 [world]");
  const int64_t* so = src_off.data_ptr<int64_t>();
  const int64_t* nb = nbytes.data_ptr<int64_t>();
  const int64_t* dof = dst_off.data_ptr<int64_t>();
  const int64_t cap = dst.numel() * dst.element_size();
  for (int p = 0; p < c.world; ++p)
    TORCH_CHECK(nb[p] >= 0 && dof[p] >= 0 && so[p] >= 0 && dof[p] + nb[p] <= cap, "xgmi pull: range of peer ", p);
  c10::DeviceGuard g(dst.device());
  hipStream_t st = cur_stream();
  fork(c, st);
  auto* d = static_cast<uint8_t*>(dst.data_ptr());
  for (int k = 1; k < c.world; ++k) {
    const int p = (c.rank + k) % c.world;
    TORCH_CHECK(c.shared[slot][p] != nullptr, "xgmi pull: peer ", p, " of slot ", slot, " not opened");
    if (nb[p] == 0) continue;
    XGMI_CHECK(hipMemcpyAsync(d + dof[p], c.shared[slot][p] + so[p], (size_t)nb[p], hipMemcpyDeviceToDevice,
                              c.peer_st[p]));
  }
  join(c, st);
}

// out = own + sum over peers p != rank of scratch[p] (bf16, f32 accumulation in rank order 0 ..
// world-1, so every rank's result does not depend on which rank computes it).  scratch is
// [world, n] (the own row unused), own and out are [n].
__global__ void reduce_rows_kernel(const u32x4* __restrict__ scratch, const u32x4* __restrict__ own,
                                   u32x4* __restrict__ out, int me, int world, int64_t n16) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x) {
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < world; ++r) {
      const u32x4 v = r == me ? own[i] : __builtin_nontemporal_load(scratch + (int64_t)r * n16 + i);
      acc8_bf16(a, v);
    }
    out[i] = pack8_bf16(a);
  }
}

void reduce_pulled(int64_t id, const at::Tensor& out, const at::Tensor& scratch, const at::Tensor& own) {
  Comm& c = get(id);
  for (const at::Tensor* t : {&out, &scratch, &own})
    TORCH_CHECK(t->is_cuda() && t->is_contiguous() && t->scalar_type() == at::kBFloat16 &&
                    reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0,
                "xgmi reduce_pulled: bf16, contiguous, 16-byte aligned");
  const int64_t n = out.numel();
  TORCH_CHECK(own.numel() == n && scratch.numel() == n * c.world && n % 8 == 0, "xgmi reduce_pulled: shapes");
  if (n == 0) return;
  c10::DeviceGuard g(out.device());
  const int64_t n16 = n / 8;
  reduce_rows_kernel<<<grid_for(n16), 256, 0, cur_stream()>>>(
      reinterpret_cast<const u32x4*>(scratch.data_ptr()), reinterpret_cast<const u32x4*>(own.data_ptr()),
      reinterpret_cast<u32x4*>(out.data_ptr()), c.rank, c.world, n16);
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

TORCH_LIBRARY(dtg_xgmi, m) {
  m.def("alloc_shared(int id, int nbytes) -> Tensor", &alloc_shared);
  m.def("shared_handle(int id, int slot) -> Tensor", &shared_handle);
  m.def("open_shared(int id, int slot, Tensor handles) -> ()", &open_shared);
  m.def("signal_wait(int id) -> ()", &signal_wait);
  m.def("pull(int id, int slot, Tensor(a!) dst, Tensor src_off, Tensor nbytes, Tensor dst_off) -> ()", &pull);
  m.def("reduce_pulled(int id, Tensor(a!) out, Tensor scratch, Tensor own) -> ()", &reduce_pulled);
  m.def("create(int capacity, int rank, int world, int device) -> int", &create);
  m.def("ipc_handle(int id) -> Tensor", &ipc_handle);
  m.def("open_peers(int id, Tensor handles) -> ()", &open_peers);
  m.def("set_timeout(int id, float seconds) -> ()", &set_timeout);
  m.def("error(int id) -> int", &error);
  m.def("destroy(int id) -> ()", &destroy);
  m.def("workspace(int id) -> Tensor", &workspace);
  m.def("workspace_view(int id, int offset, int[] sizes, ScalarType dtype) -> Tensor", &workspace_view);
  m.def("all_gather(int id, Tensor(a!) out, Tensor inp, int offset=0) -> ()", &all_gather);
  m.def("all_gather_dma(int id, Tensor(a!) out, Tensor inp, int offset=0) -> ()", &all_gather_dma);
  m.def("reduce_scatter(int id, Tensor(a!) out, Tensor inp, int offset=0) -> ()", &reduce_scatter);
  m.def("reduce_scatter_dma(int id, Tensor(a!) out, Tensor inp, int offset=0) -> ()", &reduce_scatter_dma);
  m.def("all_reduce(int id, Tensor(a!) inout, int offset=0) -> ()", &all_reduce);
}

}  // namespace xgmi
}  // namespace dtg
