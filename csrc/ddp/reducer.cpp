// Native gradient-bucket reducer for the mi355x_dp data-parallel engine (SURVEY.md §2.3 N1:
// the counterpart of torch DDP's C++ Reducer, reached by the reference through
// torch.nn.parallel.DistributedDataParallel at cifar10-distributed-smddp-gpu.py:148).
//
// The gradients of every parameter live in ONE flat fp32 buffer (mi355x_dp.parallel.flat),
// so a bucket is a contiguous slice -- no copy-in / copy-out kernels.  This object owns:
//
//  * the link-aware bucket planner: bucket sizes from an alpha-beta model of a ring
//    all-reduce over point-to-point xGMI (7 links x ~153 GB/s per MI355X): the first bucket
//    small (communication starts after the first few backward kernels), the LAST bucket
//    small (its all-reduce is the exposed tail after backward ends), the middle ones large
//    enough that the per-collective latency is <= ~10 % of the transfer;
//  * grad-ready bookkeeping: backward kernels (or post-accumulate hooks) call mark_ready(i);
//    when every parameter of the next bucket in order is ready, its all-reduce is launched
//    on the process group -- in the same order on every rank, so collectives match;
//  * the comm itself is asynchronous on the backend's side stream (RCCL / native smddp
//    backend: the collective waits on an event of the producing stream, Work::wait makes
//    the consumer stream wait on the completion event -- no host synchronisation);
//  * finish(): launch buckets whose parameters never got a gradient (unused parameters:
//    their zeroed slice is still reduced, matching DDP's find_unused_parameters=False
//    semantics where every rank participates) and wait for all outstanding work.
//  * balanced-shard mode (SMDDP's "each GPU reduces one shard of the fused buffer", SURVEY.md
//    §2.4 / §5.8): a bucket is REDUCE-SCATTERED in place instead of all-reduced -- rank r ends
//    up with the summed gradient of the r-th 1/world of every bucket, the optimizer updates only
//    that shard, and gather_params() all-gathers the updated parameter shards in place (one
//    collective per bucket).  The flat layout pads every bucket to a multiple of world x 64
//    elements so the shards are equal and aligned.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>
#include <torch/csrc/distributed/c10d/Types.hpp>
#include <torch/csrc/distributed/c10d/Work.hpp>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <tuple>
#include <map>
#include <mutex>
#include <optional>
#include <string>
#include <vector>

namespace mi_ddp {

// Ring all-reduce time model T(S) = alpha + 2 (W-1)/W * S / B.  Returns the bucket size at
// which alpha is `overhead` of T, clamped to [min_bytes, max_bytes].
int64_t link_aware_cap(int world, double link_gbps, int links, double alpha_us, double overhead, int64_t min_bytes,
                       int64_t max_bytes) {
  if (world <= 1) return max_bytes;
  // a ring uses one link per direction; RCCL runs several rings over disjoint links
  const double rings = std::max(1, std::min(links, world - 1));
  const double bw = link_gbps * 1e9 * rings;                         // bytes / s
  const double factor = 2.0 * (world - 1) / world;
  const double s = alpha_us * 1e-6 * (1.0 - overhead) / overhead * bw / factor;
  return std::max(min_bytes, std::min(max_bytes, (int64_t)s));
}

// Greedy contiguous buckets over tensors in backward order.  The first bucket is capped at
// `first`, the last at `last` (planned from the end), the rest at `cap`.  Afterwards every
// bucket smaller than `min_bytes` is merged into its successor (the tail into its predecessor):
// with parameters in reverse registration order the first bucket would otherwise be a lone
// 4 KB fc.bias -- a collective that pays the full launch latency for nothing.
std::vector<std::vector<int64_t>> merge_small(std::vector<std::vector<int64_t>> out, const std::vector<int64_t>& bytes,
                                              int64_t min_bytes) {
  auto size = [&](const std::vector<int64_t>& b) {
    int64_t s = 0;
    for (int64_t i : b) s += bytes[i];
    return s;
  };
  size_t i = 0;
  while (out.size() > 1 && i < out.size()) {
    if (size(out[i]) >= min_bytes) {
      ++i;
      continue;
    }
    if (i + 1 < out.size()) {
      out[i].insert(out[i].end(), out[i + 1].begin(), out[i + 1].end());
      out.erase(out.begin() + i + 1);
    } else {
      out[i - 1].insert(out[i - 1].end(), out[i].begin(), out[i].end());
      out.erase(out.begin() + i);
    }
  }
  return out;
}

std::vector<std::vector<int64_t>> plan_buckets(const std::vector<int64_t>& bytes, int64_t cap, int64_t first,
                                               int64_t last, int64_t min_bytes) {
  const int64_t n = (int64_t)bytes.size();
  std::vector<std::vector<int64_t>> out;
  if (n == 0) return out;
  // tail bucket: the trailing tensors up to `last` bytes (at least one)
  int64_t tail_begin = n - 1, acc = bytes[n - 1];
  while (tail_begin > 0 && acc + bytes[tail_begin - 1] <= last) acc += bytes[--tail_begin];
  std::vector<int64_t> cur;
  int64_t cur_bytes = 0, lim = first;
  for (int64_t i = 0; i < tail_begin; ++i) {
    // a bucket is closed only once it holds >= min_bytes: a first bucket capped below the
    // first large tensor takes that tensor instead of leaving a sliver in front of it
    if (!cur.empty() && cur_bytes + bytes[i] > lim && cur_bytes >= min_bytes) {
      out.push_back(cur);
      cur.clear();
      cur_bytes = 0;
      lim = cap;
    }
    cur.push_back(i);
    cur_bytes += bytes[i];
  }
  if (!cur.empty()) out.push_back(cur);
  std::vector<int64_t> tail;
  for (int64_t i = tail_begin; i < n; ++i) tail.push_back(i);
  out.push_back(tail);
  return merge_small(std::move(out), bytes, min_bytes);
}

class Reducer {
 public:
  Reducer(at::Tensor flat_grad, std::vector<int64_t> offsets, std::vector<int64_t> numels,
          std::vector<std::vector<int64_t>> buckets, c10::intrusive_ptr<c10d::ProcessGroup> pg, int64_t align,
          bool force_comm, c10::optional<at::Tensor> comm_buf, bool shard)
      : grad_(std::move(flat_grad)), offsets_(std::move(offsets)), numels_(std::move(numels)),
        buckets_(std::move(buckets)), pg_(std::move(pg)), force_comm_(force_comm), shard_(shard) {
    TORCH_CHECK(offsets_.size() == numels_.size(), "offsets / numels mismatch");
    if (comm_buf.has_value() && comm_buf->defined()) {
      // reduced-precision gradient exchange: each bucket is cast into this buffer on the producing
      // stream, all-reduced there (half the bytes over xGMI for bf16), and cast back into the fp32
      // gradient in finish() -- every rank receives the identical reduced values, so replicas stay
      // bit-identical; the fp32 master weights and optimizer are unchanged
      comm_ = *comm_buf;
      TORCH_CHECK(comm_.numel() >= grad_.numel() && comm_.device() == grad_.device(), "bad comm buffer");
    }
    const int64_t np = (int64_t)offsets_.size();
    bucket_of_.assign(np, -1);
    for (size_t b = 0; b < buckets_.size(); ++b) {
      TORCH_CHECK(!buckets_[b].empty(), "empty bucket");
      int64_t lo = INT64_MAX, hi = 0;
      for (int64_t i : buckets_[b]) {
        TORCH_CHECK(i >= 0 && i < np && bucket_of_[i] < 0, "bad bucket plan");
        bucket_of_[i] = (int64_t)b;
        lo = std::min(lo, offsets_[i]);
        hi = std::max(hi, offsets_[i] + numels_[i]);
      }
      hi = std::min(grad_.numel(), (hi + align - 1) / align * align);
      ranges_.emplace_back(lo, hi);
    }
    for (int64_t i = 0; i < np; ++i) TORCH_CHECK(bucket_of_[i] >= 0, "parameter ", i, " not in any bucket");
    if (shard_) {
      world_ = pg_ ? pg_->getSize() : 1;
      rank_ = pg_ ? pg_->getRank() : 0;
      for (const auto& r : ranges_)
        TORCH_CHECK((r.second - r.first) % world_ == 0, "shard mode: bucket [", r.first, ", ", r.second,
                    ") is not a multiple of world size ", world_, " (pad the flat layout per bucket)");
    }
    reset();
  }

  ~Reducer() {
    for (auto* v : {&ev_ready_, &ev_end_})
      for (hipEvent_t e : *v) hipEventDestroy(e);
    if (ev_t0_) hipEventDestroy(ev_t0_);
    if (ev_bwd_end_) hipEventDestroy(ev_bwd_end_);
  }

  // GPU-side timeline of the bucket collectives (host launch times are not
  // overlap evidence).  Per step, relative to an event recorded on the current stream at reset()
  // (the forward's start): `ready` = an event on the producing stream just before the bucket's
  // collective is issued (its gradients -- and a bf16 cast -- are complete there), `end` = an event
  // on a probe stream made to wait on the collective's Work (the collective's completion), and
  // `bwd_end` = an event on the current stream when finish() starts (the compute stream has joined
  // the weight-gradient stream there: the end of the backward's kernels).  Collectives are serial on
  // the comm stream, so each one starts at max(its ready, the previous end).  Not recorded inside a
  // graph capture.
  void set_gpu_timing(bool on) {
    std::lock_guard<std::mutex> g(mu_);
    if (on && !grad_.is_cuda()) return;
    timing_ = on;
    if (!on || !ev_ready_.empty()) return;
    c10::hip::HIPGuardMasqueradingAsCUDA dg(grad_.device());
    ev_ready_.assign(buckets_.size(), nullptr);
    ev_end_.assign(buckets_.size(), nullptr);
    for (auto* v : {&ev_ready_, &ev_end_})
      for (auto& e : *v) TORCH_CHECK(hipEventCreate(&e) == hipSuccess, "hipEventCreate");
    TORCH_CHECK(hipEventCreate(&ev_t0_) == hipSuccess && hipEventCreate(&ev_bwd_end_) == hipSuccess, "hipEventCreate");
    probe_ = c10::hip::getStreamFromPoolMasqueradingAsCUDA(true, grad_.device().index());
  }
  bool gpu_timing() const { return timing_; }

  // {"bwd_end_ms": ..} plus per launched bucket (b, bytes, ready_ms, end_ms) of the last step;
  // synchronises on the step's last events (call after the step, never inside the timed loop)
  std::pair<double, std::vector<std::tuple<int64_t, int64_t, double, double>>> gpu_trace() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<std::tuple<int64_t, int64_t, double, double>> out;
    if (!timing_ || !t0_ok_) return {-1.0, out};
    auto ms = [&](hipEvent_t e) {
      float v = -1.f;
      if (hipEventSynchronize(e) != hipSuccess || hipEventElapsedTime(&v, ev_t0_, e) != hipSuccess) return -1.0;
      return (double)v;
    };
    for (size_t b = 0; b < timed_.size(); ++b)
      if (timed_[b]) {
        const auto& r = ranges_[b];
        const int64_t esz = comm_.defined() ? comm_.element_size() : grad_.element_size();
        out.emplace_back((int64_t)b, (r.second - r.first) * esz, ms(ev_ready_[b]), ms(ev_end_[b]));
      }
    return {bwd_end_ok_ ? ms(ev_bwd_end_) : -1.0, out};
  }

  void reset() {
    std::lock_guard<std::mutex> g(mu_);
    timed_.assign(buckets_.size(), false);
    t0_ok_ = bwd_end_ok_ = false;
    if (timing_) {
      auto cur = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(grad_.device().index());
      if (!capturing(cur.stream())) t0_ok_ = hipEventRecord(ev_t0_, cur.stream()) == hipSuccess;
    }
    pending_.assign(buckets_.size(), 0);
    for (size_t b = 0; b < buckets_.size(); ++b) pending_[b] = (int64_t)buckets_[b].size();
    ready_.assign(buckets_.size(), false);
    param_ready_.assign(offsets_.size(), false);
    works_.clear();
    next_ = 0;
    sent_.assign(buckets_.size(), false);
    trace_.clear();
    t0_ = std::chrono::steady_clock::now();
  }

  // DDP no_sync(): while disabled, gradients only accumulate locally -- no bucket is launched
  // and finish() returns at once; the next synchronised backward reduces the accumulated sums
  void set_enabled(bool on) {
    std::lock_guard<std::mutex> g(mu_);
    enabled_ = on;
  }
  bool enabled() const { return enabled_; }

  void mark_ready(int64_t i) {
    std::lock_guard<std::mutex> g(mu_);
    if (!enabled_) return;
    TORCH_CHECK(i >= 0 && i < (int64_t)param_ready_.size(), "parameter index out of range");
    if (param_ready_[i]) return;
    param_ready_[i] = true;
    const int64_t b = bucket_of_[i];
    if (--pending_[b] == 0) {
      ready_[b] = true;
      launch_ready_locked();
    }
  }

  void finish() {
    std::vector<c10::intrusive_ptr<c10d::Work>> works;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!enabled_) return;
      std::fill(ready_.begin(), ready_.end(), true);
      launch_ready_locked();
      works.swap(works_);
      if (timing_ && t0_ok_ && !works.empty()) {
        auto cur = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(grad_.device().index());
        if (!capturing(cur.stream())) bwd_end_ok_ = hipEventRecord(ev_bwd_end_, cur.stream()) == hipSuccess;
      }
    }
    for (auto& w : works) w->wait();
    std::lock_guard<std::mutex> g(mu_);
    if (comm_.defined())
      for (int64_t b = 0; b < (int64_t)ranges_.size(); ++b)
        if (sent_[b]) {
          const auto sh = shard_range(b);
          grad_.narrow(0, sh.first, sh.second - sh.first).copy_(comm_.narrow(0, sh.first, sh.second - sh.first));
        }
    trace_.emplace_back(-1, 0, since_reset_us());
  }

  // [lo, hi) of this rank's shard of bucket b (the whole bucket when not sharding)
  std::pair<int64_t, int64_t> shard_range(int64_t b) const {
    const auto& r = ranges_[b];
    if (!shard_) return r;
    const int64_t c = (r.second - r.first) / world_;
    return {r.first + rank_ * c, r.first + (rank_ + 1) * c};
  }

  // shard mode, after the optimizer updated this rank's shards of `params` (same layout as the
  // gradient buffer): all-gather every bucket in place, in bucket order, on the backend's stream
  // (ordered after the optimizer kernel through the producing-stream event); wait_gather() makes
  // the caller's stream wait for them -- no host synchronisation
  void gather_params(at::Tensor params) {
    std::lock_guard<std::mutex> g(mu_);
    TORCH_CHECK(shard_, "gather_params: reducer not in shard mode");
    TORCH_CHECK(params.numel() == grad_.numel() && params.device() == grad_.device(), "gather_params: bad buffer");
    if (!pg_ || !(pg_->getSize() > 1 || force_comm_)) return;
    for (int64_t b = 0; b < (int64_t)ranges_.size(); ++b) {
      const auto& r = ranges_[b];
      const auto sh = shard_range(b);
      at::Tensor whole = params.narrow(0, r.first, r.second - r.first);
      at::Tensor mine = params.narrow(0, sh.first, sh.second - sh.first);
      gather_works_.push_back(pg_->_allgather_base(whole, mine, c10d::AllgatherOptions()));
      ++comm_calls_;
      comm_bytes_ += (r.second - r.first) * params.element_size();
    }
  }

  void wait_gather() {
    std::vector<c10::intrusive_ptr<c10d::Work>> works;
    {
      std::lock_guard<std::mutex> g(mu_);
      works.swap(gather_works_);
    }
    for (auto& w : works) w->wait();
  }

  bool sharded() const { return shard_; }

  int64_t num_buckets() const { return (int64_t)buckets_.size(); }
  int64_t launched() const { return next_; }
  int64_t comm_calls() const { return comm_calls_; }
  int64_t comm_bytes() const { return comm_bytes_; }
  std::vector<std::pair<int64_t, int64_t>> ranges() const { return ranges_; }
  std::vector<std::vector<int64_t>> buckets() const { return buckets_; }
  // (bucket, bytes, host launch time in us since reset()) of every bucket of the current step,
  // in launch order; finish() appends (-1, 0, time all collectives were waited on)
  std::vector<std::tuple<int64_t, int64_t, double>> trace() {
    std::lock_guard<std::mutex> g(mu_);
    return trace_;
  }

 private:
  static bool capturing(hipStream_t s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
  }

  double since_reset_us() const {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0_).count();
  }

  void launch_ready_locked() {
    while (next_ < (int64_t)buckets_.size() && ready_[next_]) {
      const auto& r = ranges_[next_];
      const at::Tensor& buf = comm_.defined() ? comm_ : grad_;
      trace_.emplace_back(next_, (r.second - r.first) * buf.element_size(), since_reset_us());
      if (pg_ && (pg_->getSize() > 1 || force_comm_)) {
        // GPU timeline only outside a capture: inside one the event would be a captured node and
        // the probe stream (never captured) would wait on a captured Work
        hipStream_t cur_s = nullptr;
        bool timed = timing_ && t0_ok_;
        if (timed) {
          cur_s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(grad_.device().index()).stream();
          timed = !capturing(cur_s);
          if (timed) hipEventRecord(ev_ready_[next_], cur_s);
        }
        at::Tensor slice = grad_.narrow(0, r.first, r.second - r.first);
        if (comm_.defined()) {
          at::Tensor c = comm_.narrow(0, r.first, r.second - r.first);
          c.copy_(slice);  // cast on the caller's (producing) stream, ordered before the collective
          slice = c;
          sent_[next_] = true;
        }
        if (shard_) {
          // in place: this rank's shard of the slice receives the sum of every rank's shard
          const int64_t c = slice.numel() / world_;
          at::Tensor out = slice.narrow(0, rank_ * c, c);
          c10d::ReduceScatterOptions opts;
          opts.reduceOp = c10d::ReduceOp::SUM;
          works_.push_back(pg_->_reduce_scatter_base(out, slice, opts));
        } else {
          std::vector<at::Tensor> ts{slice};
          c10d::AllreduceOptions opts;
          opts.reduceOp = c10d::ReduceOp::SUM;
          works_.push_back(pg_->allreduce(ts, opts));
        }
        if (timed) {
          // the probe stream waits on the collective (Work::wait is a stream wait), then records
          c10::hip::HIPStreamGuardMasqueradingAsCUDA pg_guard(*probe_);
          works_.back()->wait();
          timed_[next_] = hipEventRecord(ev_end_[next_], probe_->stream()) == hipSuccess;
        }
        ++comm_calls_;
        comm_bytes_ += (r.second - r.first) * slice.element_size();
      }
      ++next_;
    }
  }

  at::Tensor grad_;
  std::vector<int64_t> offsets_, numels_;
  std::vector<std::vector<int64_t>> buckets_;
  c10::intrusive_ptr<c10d::ProcessGroup> pg_;
  std::vector<std::pair<int64_t, int64_t>> ranges_;
  std::vector<int64_t> bucket_of_, pending_;
  std::vector<bool> ready_, param_ready_, sent_;
  at::Tensor comm_;
  std::vector<c10::intrusive_ptr<c10d::Work>> works_, gather_works_;
  bool force_comm_ = false, shard_ = false, enabled_ = true;
  int64_t world_ = 1, rank_ = 0;
  std::vector<std::tuple<int64_t, int64_t, double>> trace_;
  std::chrono::steady_clock::time_point t0_ = std::chrono::steady_clock::now();
  int64_t next_ = 0, comm_calls_ = 0, comm_bytes_ = 0;
  // GPU timeline (set_gpu_timing)
  bool timing_ = false, t0_ok_ = false, bwd_end_ok_ = false;
  std::vector<hipEvent_t> ev_ready_, ev_end_;
  std::vector<bool> timed_;
  hipEvent_t ev_t0_ = nullptr, ev_bwd_end_ = nullptr;
  std::optional<c10::hip::HIPStreamMasqueradingAsCUDA> probe_;
  std::mutex mu_;
};

}  // namespace mi_ddp

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  namespace py = pybind11;
  m.doc() = "mi355x_dp native gradient-bucket reducer";
  m.def("link_aware_cap", &mi_ddp::link_aware_cap, py::arg("world"), py::arg("link_gbps") = 153.0,
        py::arg("links") = 7, py::arg("alpha_us") = 25.0, py::arg("overhead") = 0.1,
        py::arg("min_bytes") = int64_t(4) << 20, py::arg("max_bytes") = int64_t(32) << 20);
  m.def("plan_buckets", &mi_ddp::plan_buckets, py::arg("bytes"), py::arg("cap"), py::arg("first"), py::arg("last"),
        py::arg("min_bytes") = 0);
  py::class_<mi_ddp::Reducer>(m, "Reducer")
      .def(py::init<at::Tensor, std::vector<int64_t>, std::vector<int64_t>, std::vector<std::vector<int64_t>>,
                    c10::intrusive_ptr<c10d::ProcessGroup>, int64_t, bool, c10::optional<at::Tensor>, bool>(),
           py::arg("flat_grad"), py::arg("offsets"), py::arg("numels"), py::arg("buckets"), py::arg("process_group"),
           py::arg("align") = 64, py::arg("force_comm") = false, py::arg("comm_buf") = py::none(),
           py::arg("shard") = false)
      .def("reset", &mi_ddp::Reducer::reset)
      .def("mark_ready", &mi_ddp::Reducer::mark_ready, py::call_guard<py::gil_scoped_release>())
      .def("finish", &mi_ddp::Reducer::finish, py::call_guard<py::gil_scoped_release>())
      .def("shard_range", &mi_ddp::Reducer::shard_range)
      .def("gather_params", &mi_ddp::Reducer::gather_params, py::call_guard<py::gil_scoped_release>())
      .def("wait_gather", &mi_ddp::Reducer::wait_gather, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("sharded", &mi_ddp::Reducer::sharded)
      .def_property("enabled", &mi_ddp::Reducer::enabled, &mi_ddp::Reducer::set_enabled)
      .def_property_readonly("num_buckets", &mi_ddp::Reducer::num_buckets)
      .def_property_readonly("launched", &mi_ddp::Reducer::launched)
      .def_property_readonly("comm_calls", &mi_ddp::Reducer::comm_calls)
      .def_property_readonly("comm_bytes", &mi_ddp::Reducer::comm_bytes)
      .def_property_readonly("ranges", &mi_ddp::Reducer::ranges)
      .def_property_readonly("buckets", &mi_ddp::Reducer::buckets)
      .def_property_readonly("trace", &mi_ddp::Reducer::trace)
      .def_property("gpu_timing", &mi_ddp::Reducer::gpu_timing, &mi_ddp::Reducer::set_gpu_timing)
      .def("gpu_trace", &mi_ddp::Reducer::gpu_trace, py::call_guard<py::gil_scoped_release>());
}
