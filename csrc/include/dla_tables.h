// Device-resident tensor tables shared between the op bindings and the comm engine.
#pragma once
#include <torch/extension.h>
#include <vector>
#include "dla_kernels.h"

namespace dla {

int dtype_code(const at::Tensor& t);
hipStream_t current_stream(const at::Tensor& t);
void check_dev(const at::Tensor& t, const char* what);
// Same element order in memory: equal shapes and equal strides on every dimension of size > 1
// (the strides of size-1 dimensions are arbitrary, e.g. 1x1 conv weights in channels_last).
inline bool same_layout(const at::Tensor& a, const at::Tensor& b) {
  if (a.sizes() != b.sizes()) return false;
  for (int64_t d = 0; d < a.dim(); ++d)
    if (a.size(d) > 1 && a.stride(d) != b.stride(d)) return false;
  return true;
}
at::Tensor upload(const void* data, size_t bytes, const at::Device& dev);
// Gathers `ts` into `flat` at element offsets `offs` on stream `st` (by-value list launches).
void pack_tensors_on(const std::vector<at::Tensor>& ts, const std::vector<int64_t>& offs, const at::Tensor& flat,
                     float scale, hipStream_t st);

// PackTable: gathers a bucket's gradients into a flat buffer (tensor fusion) and scatters the
// reduced buffer back, each as ONE multi-tensor launch (csrc/kernels/multi_tensor.hip).
class PackTable {
 public:
  PackTable(std::vector<at::Tensor> tensors, std::vector<int64_t> offsets) : tensors_(std::move(tensors)) {
    TORCH_CHECK(tensors_.size() == offsets.size(), "PackTable: tensors/offsets size mismatch");
    TORCH_CHECK(!tensors_.empty(), "PackTable: empty tensor list");
    dtype_ = dtype_code(tensors_[0]);
    std::vector<PackEntry> entries;
    std::vector<int32_t> prefix;
    int32_t blocks = 0;
    const int chunk = mt_chunk_elems();
    for (size_t i = 0; i < tensors_.size(); ++i) {
      check_dev(tensors_[i], "bucket tensor");
      TORCH_CHECK(dtype_code(tensors_[i]) == dtype_, "PackTable: all tensors must share a dtype");
      PackEntry e{tensors_[i].data_ptr(), tensors_[i].numel(), offsets[i]};
      total_ = std::max(total_, offsets[i] + e.numel);
      if (e.numel == 0) continue;
      entries.push_back(e);
      prefix.push_back(blocks);
      blocks += (int32_t)((e.numel + chunk - 1) / chunk);
    }
    ntensors_ = (int)entries.size();
    nblocks_ = blocks;
    entries_ = upload(entries.data(), entries.size() * sizeof(PackEntry), tensors_[0].device());
    prefix_ = upload(prefix.data(), prefix.size() * sizeof(int32_t), tensors_[0].device());
  }

  void pack(at::Tensor flat, double scale) {
    check_dev(flat, "flat");
    TORCH_CHECK(flat.numel() >= total_, "PackTable.pack: flat buffer too small");
    launch_pack(reinterpret_cast<const PackEntry*>(entries_.data_ptr()), reinterpret_cast<const int32_t*>(prefix_.data_ptr()), ntensors_,
                nblocks_, dtype_, dtype_code(flat), flat.data_ptr(), (float)scale, current_stream(flat));
  }

  void unpack(at::Tensor flat, double scale) {
    check_dev(flat, "flat");
    TORCH_CHECK(flat.numel() >= total_, "PackTable.unpack: flat buffer too small");
    launch_unpack(reinterpret_cast<const PackEntry*>(entries_.data_ptr()), reinterpret_cast<const int32_t*>(prefix_.data_ptr()), ntensors_,
                  nblocks_, dtype_code(flat), dtype_, flat.data_ptr(), (float)scale, current_stream(flat));
  }

  // Launches pack/unpack on an explicit stream (used by the comm engine).
  void pack_on(at::Tensor flat, double scale, hipStream_t s) {
    launch_pack(reinterpret_cast<const PackEntry*>(entries_.data_ptr()), reinterpret_cast<const int32_t*>(prefix_.data_ptr()), ntensors_,
                nblocks_, dtype_, dtype_code(flat), flat.data_ptr(), (float)scale, s);
  }
  void unpack_on(at::Tensor flat, double scale, hipStream_t s) {
    launch_unpack(reinterpret_cast<const PackEntry*>(entries_.data_ptr()), reinterpret_cast<const int32_t*>(prefix_.data_ptr()), ntensors_,
                  nblocks_, dtype_code(flat), dtype_, flat.data_ptr(), (float)scale, s);
  }

  int64_t total_numel() const { return total_; }

 private:
  std::vector<at::Tensor> tensors_;
  at::Tensor entries_, prefix_;
  int ntensors_ = 0, nblocks_ = 0, dtype_ = kF32;
  int64_t total_ = 0;
};


}  // namespace dla
