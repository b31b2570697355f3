// Device-resident data path: the training batches come from a uint8 image bank that lives in HBM for the whole
// run (CIFAR-10 is 150 MB of a 288 GB device), so a step reads B images from HBM instead of decoding, augmenting
// and copying them on host worker processes (reference: datasets/base_dataset.py:96-128 transforms,
// train.py:107-128 DataLoader(pin_memory, num_workers=4)).
//
// One launch per batch: gather by index, RandomHorizontalFlip (counter-hash draw per epoch position),
// ToTensor (u / 255) and Normalize ((v - mean) / std) in the op order torchvision uses, NCHW fp32 out. Built with
// -ffp-contract=off: the division and subtraction are the correctly rounded IEEE ops of the CPU path, so the
// output equals torchvision's bit for bit.
#include "dmc_common.h"
#include "dmc_internal.h"

namespace {

struct Norm4 {
  float mean[4], std[4];
};

__global__ __launch_bounds__(256) void load_batch_kernel(const uint8_t* __restrict__ bank, int H, int W, int C,
                                                         const int32_t* __restrict__ idx, const uint8_t* flips,
                                                         uint32_t flip_seed, uint32_t flip_thresh, long pos0,
                                                         Norm4 nm, float* __restrict__ out,
                                                         const int64_t* labels_in, int64_t* labels_out) {
  const int b = blockIdx.x;
  const long img = idx[b];
  const int HW = H * W;
  bool flip;
  if (flips)
    flip = flips[b] != 0;
  else
    flip = flip_thresh != 0u && hash_u32((uint32_t)(pos0 + b), flip_seed) < flip_thresh;
  if (labels_out && threadIdx.x == 0) labels_out[b] = labels_in[img];
  const uint8_t* src = bank + img * (long)HW * C;
  float* dst = out + (long)b * C * HW;
  // output-contiguous walk (NCHW); the source row of one image (W*C bytes) stays in L1 for the row's threads
  for (int e = threadIdx.x; e < C * HW; e += blockDim.x) {
    const int c = e / HW, p = e - c * HW;
    const int y = p / W, x = p - y * W;
    const int sx = flip ? W - 1 - x : x;
    const float u = (float)src[(y * W + sx) * C + c];
    const float v = u / 255.0f;                 // ToTensor: img.float().div(255)
    dst[e] = (v - nm.mean[c]) / nm.std[c];      // Normalize: tensor.sub_(mean).div_(std)
  }
}

}  // namespace

extern "C" int dmc_load_batch(const uint8_t* bank, long n_images, int H, int W, int C, const int32_t* idx, int B,
                              const uint8_t* flips, uint32_t flip_seed, uint32_t flip_thresh, long pos0,
                              const float* mean, const float* std, float* out, const int64_t* labels_in,
                              int64_t* labels_out, void* stream) {
  if (B <= 0) return 0;   // empty batch: nothing to read (its pointers may be NULL)
  DMC_REQUIRE(bank && idx && out && mean && std, "dmc_load_batch: null pointer");
  DMC_REQUIRE(C >= 1 && C <= 4 && H > 0 && W > 0 && n_images > 0, "dmc_load_batch: bad image shape %dx%dx%d", H, W,
              C);
  DMC_REQUIRE((labels_in == nullptr) == (labels_out == nullptr), "dmc_load_batch: labels_in/labels_out go together");
  Norm4 nm;
  for (int c = 0; c < 4; ++c) {
    nm.mean[c] = c < C ? mean[c] : 0.f;
    nm.std[c] = c < C ? std[c] : 1.f;
    DMC_REQUIRE(nm.std[c] != 0.f, "dmc_load_batch: std[%d] is zero", c);
  }
  load_batch_kernel<<<B, 256, 0, dmc::as_stream(stream)>>>(bank, H, W, C, idx, flips, flip_seed, flip_thresh, pos0, nm,
                                                          out, labels_in, labels_out);
  return dmc::check_launch("dmc_load_batch");
}
