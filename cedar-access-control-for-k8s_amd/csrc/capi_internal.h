// Internal state behind the C-ABI handles (include/cedargpu.h), shared by capi.cpp and queue.cpp.
#pragma once
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/cedargpu.h"
#include "device.h"
#include "engine.h"

namespace cg {
struct LoadedImage {
  std::shared_ptr<Image> host;
  DevImage dev;
  ~LoadedImage() { dev_image_free(&dev); }
};

#define GUARD(errstr, body)                                       \
  try {                                                           \
    body                                                          \
  } catch (const CedarError& e) {                                 \
    errstr = e.what();                                            \
    return CG_E_PARSE;                                            \
  } catch (const std::bad_alloc&) {                               \
    errstr = "out of host memory";                                \
    return CG_E_ARG;                                              \
  } catch (const std::exception& e) {                             \
    errstr = e.what();                                            \
    return CG_E_ARG;                                              \
  }

}  // namespace cg

using cg::LoadedImage;

struct cg_ctx {
  int device = 0;
  void* stream = nullptr;
  cg::DevPool* pool = nullptr;  // batch buffers (device + pinned staging), reused across batches
  std::mutex mu;
  std::map<uint64_t, std::shared_ptr<LoadedImage>> images;
  std::shared_ptr<LoadedImage> active;
  std::string err;
  // many-hit share (RF_BIG requests per million) of the last batch that ran the on-device
  // follow-up, and the image it ran on: the next batch on that image sizes its follow-up by it
  std::atomic<uint32_t> big_ppm{0}, big_maxr{0};  // share, and the most reasons one entry needed
  std::atomic<const LoadedImage*> big_img{nullptr};
};

struct cg_batch {
  cg_ctx* ctx = nullptr;
  std::shared_ptr<LoadedImage> img;
  cg::Batch host;
  cg::DevBatch dev;
  bool submitted = false, done = false;
  uint32_t n_rerun = 0;  // requests re-run by cg_batch_wait
  std::string err;
  // items: caller-visible entries; dev >= 0 is the device request index, else a fast-path result
  struct Item { int32_t dev; int32_t fast; };
  std::vector<Item> items;
  std::map<uint32_t, std::string> fast_reason;  // authz fast paths: the reason; admission: error text
  std::vector<cg::DevSubset> held;  // re-run result blocks the host lists point into (Batch::big)
  ~cg_batch() {
    for (auto& j : held) dev_subset_release(&j);
    dev_batch_free(&dev);
  }
  int32_t dev_of(uint32_t i) const { return i < items.size() ? items[i].dev : -1; }
};

