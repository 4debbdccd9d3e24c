// wire_capi.cpp — C entry points of the wire-codec oracle (liboraclewire.so).
// TEST INFRASTRUCTURE ONLY (see wire_oracle.hpp): loaded by tests/ and by the
// cpu_baseline leg of tools/bench_wire.py, never by the product.
//
// grwo_decode / grwo_encode have exactly the contract of grw_decode / grw_encode
// (include/gpuraft_wire.h), so a test can run both on the same arrays.
#include <chrono>
#include <thread>
#include <vector>

#include "wire_oracle.hpp"

using namespace wire_oracle;

extern "C" {

int grwo_decode(const uint8_t* buf, size_t buf_len, grw_batch* batches, size_t n, grw_message* msgs,
                size_t msg_cap, grw_entry* ents, size_t ent_cap, size_t* n_msgs, size_t* n_ents) {
  for (size_t b = 0; b < n; ++b)
    if (batches[b].frame_off + batches[b].frame_len > buf_len) return -1;  // GR_EINVAL
  std::vector<grw_message> vm;
  std::vector<grw_entry> ve;
  for (size_t b = 0; b < n; ++b) batch_unmarshal(buf, batches[b], vm, ve, (uint32_t)b);
  *n_msgs = vm.size();
  *n_ents = ve.size();
  if (vm.size() > msg_cap || ve.size() > ent_cap) return -5;  // GR_ECAPACITY
  if (!vm.empty()) memcpy(msgs, vm.data(), vm.size() * sizeof(grw_message));
  if (!ve.empty()) memcpy(ents, ve.data(), ve.size() * sizeof(grw_entry));
  return 0;
}

int grwo_encode(const uint8_t* payload, size_t payload_len, grw_batch* batches, size_t n,
                const grw_message* msgs, size_t n_msgs, const grw_entry* ents, size_t n_ents, uint8_t* out,
                size_t out_cap, size_t* out_len) {
  (void)payload_len;
  (void)n_ents;
  size_t total = 0;
  for (size_t b = 0; b < n; ++b) {
    if ((size_t)batches[b].first_msg + batches[b].n_msgs > n_msgs) return -1;
    i64 s = batch_size(batches[b], msgs, ents);
    batches[b].status = s < 0 ? GRW_E_PANIC : GRW_OK;
    batches[b].frame_off = total;
    batches[b].frame_len = s < 0 ? 0 : (uint32_t)s;
    total += batches[b].frame_len;
  }
  *out_len = total;
  if (total > out_cap) return -5;
  for (size_t b = 0; b < n; ++b)
    if (batches[b].status == GRW_OK) batch_marshal(out, batches[b].frame_off, batches[b], msgs, ents, payload);
  return 0;
}

// CPU baseline: MessageBatch.Unmarshal of every frame, frames split over
// `threads` workers (each with its own record vectors, as each Go transport
// goroutine unmarshals into its own batch), repeated until `seconds` elapse.
// Returns messages decoded per second; *reps_out = passes completed.
double grwo_decode_bench(const uint8_t* buf, const grw_batch* batches, size_t n, int threads, double seconds,
                         uint64_t* reps_out) {
  using clk = std::chrono::steady_clock;
  std::vector<uint64_t> msgs_done(threads, 0);
  auto t0 = clk::now();
  uint64_t reps = 0;
  while (true) {
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t) {
      ts.emplace_back([&, t]() {
        std::vector<grw_message> vm;
        std::vector<grw_entry> ve;
        for (size_t b = (size_t)t; b < n; b += (size_t)threads) {
          grw_batch bb = batches[b];
          vm.clear();
          ve.clear();
          batch_unmarshal(buf, bb, vm, ve, (uint32_t)b);
          msgs_done[t] += vm.size();
        }
      });
    }
    for (auto& th : ts) th.join();
    reps++;
    double el = std::chrono::duration<double>(clk::now() - t0).count();
    if (el >= seconds) {
      uint64_t tot = 0;
      for (auto v : msgs_done) tot += v;
      *reps_out = reps;
      return (double)tot / el;
    }
  }
}

}  // extern "C"
