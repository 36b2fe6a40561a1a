// capture.cpp — the dataset capture pipeline of Engine::captureSceneData (Vulkan_Engine/engine.cpp:
// 2658-2814) on the C-ABI: per view, accumulation_steps samples in ONE
// ptgs_trace_camera call, sRGB8 encode, read-back, every-2nd-pixel downscale, JPEG q90; the
// transforms JSON splits and the points3d.ply point cloud. The host-only pieces (poses, glm::inverse,
// the JSON number printer and the writers) are in capture_io.cpp.
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <vector>

#include "../../include/ptgs/ptgs.h"
#include "../../include/ptgs/ptgs_host.h"

bool ptgs_mkdirs(const std::string& path);  // capture_io.cpp

extern "C" {

int ptgs_capture_dataset(ptgs_ctx* ctx, const ptgs_capture_desc* d) {
  if (!ctx || !d || !d->out_dir || !d->ubo) return PTGS_EINVAL;
  if (d->width == 0 || d->height == 0) return PTGS_EINVAL;
  if (d->capture_pointcloud && (!d->samples || d->num_samples == 0)) return PTGS_EINVAL;
  const std::string root = d->out_dir;
  if (!ptgs_mkdirs(root + "/train")) return PTGS_EIO;
  const uint32_t W = d->width, H = d->height;
  const float aspect = (float)W / (float)H;
  hipStream_t s = (hipStream_t)d->hip_stream;
  int rc = PTGS_OK;
  float* accum = nullptr;
  uint32_t* rgba8 = nullptr;
  std::vector<uint32_t> host((size_t)W * H);
  std::vector<float> transforms_train, transforms_test;
  std::vector<std::string> paths_train, paths_test;
  if (d->capture_images) {
    if ((rc = ptgs_device_alloc(ctx, (size_t)W * H * 16, (void**)&accum))) return rc;
    if ((rc = ptgs_device_alloc(ctx, (size_t)W * H * 4, (void**)&rgba8))) {
      ptgs_device_free(ctx, accum);
      return rc;
    }
    std::vector<float> ab(2 * (size_t)d->total_positions);
    ptgs_capture_poses(d->total_positions, d->seed, d->min_beta, d->max_beta, ab.data());
    for (uint32_t i = 0; i < d->total_positions && rc == PTGS_OK; ++i) {
      ptgs_ubo ubo = *d->ubo;
      float pos[3];
      ptgs_camera_toroidal(ab[2 * i], ab[2 * i + 1], d->major_radius, d->torus_height, d->fov_deg, aspect, 0.1f,
                           10000.0f, ubo.view, ubo.proj, pos);
      std::memcpy(ubo.camera_pos, pos, sizeof(pos));
      ubo.frame_count = 0;
      ubo.fov = d->fov_deg * 0.01745329251994329576923690768489f;
      ubo.height = (float)H;
      if ((rc = ptgs_trace_camera(ctx, &ubo, W, H, accum, d->accumulation_steps, 1, PTGS_ACCUM_RUNNING_MEAN, s)))
        break;
      if ((rc = ptgs_encode_srgb8(ctx, accum, W, H, rgba8, s))) break;
      if (hipMemcpyAsync(host.data(), rgba8, host.size() * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess) {
        rc = PTGS_EHIP;
        break;
      }
      // :2737-2754 — every 2nd pixel of every 2nd row, alpha 255 (the stride is 2 whatever the divisor)
      uint32_t tw = W, th = H;
      std::vector<uint8_t> rgb;
      const uint8_t* px = reinterpret_cast<const uint8_t*>(host.data());
      if (d->image_divisor > 1.0f) {
        tw = (uint32_t)((float)W / d->image_divisor);
        th = (uint32_t)((float)H / d->image_divisor);
        rgb.resize((size_t)tw * th * 4);
        for (uint32_t y = 0; y < th; ++y)
          for (uint32_t x = 0; x < tw; ++x) {
            const uint8_t* sp = px + ((size_t)(y * 2) * W + x * 2) * 4;
            uint8_t* dp = rgb.data() + ((size_t)y * tw + x) * 4;
            dp[0] = sp[0];
            dp[1] = sp[1];
            dp[2] = sp[2];
            dp[3] = 255;
          }
        px = rgb.data();
      }
      const std::string rel = "train/r_" + std::to_string(i);
      if ((rc = ptgs_write_jpeg((root + "/" + rel + ".jpg").c_str(), px, tw, th, 4, 90))) break;
      float inv[16];
      ptgs_mat4_inverse_glm(ubo.view, inv);
      std::vector<float>& T = (i % 4 == 0) ? transforms_test : transforms_train;
      (i % 4 == 0 ? paths_test : paths_train).push_back("./" + rel);
      T.insert(T.end(), inv, inv + 16);
    }
    ptgs_device_free(ctx, accum);
    ptgs_device_free(ctx, rgba8);
    if (rc) return rc;
  }
  uint32_t npoints = 0;
  if (d->capture_pointcloud) {
    ptgs_hitdata* hits = nullptr;
    if ((rc = ptgs_device_alloc(ctx, (size_t)d->num_samples * sizeof(ptgs_hitdata), (void**)&hits))) return rc;
    for (uint32_t frame = 0; frame < d->accumulation_steps && rc == PTGS_OK; ++frame) {
      ptgs_ubo ubo = *d->ubo;
      ubo.frame_count = frame;
      rc = ptgs_trace_torus(ctx, &ubo, &d->torus, d->samples, d->num_samples, hits, s);
    }
    std::vector<ptgs_hitdata> h(d->num_samples);
    if (rc == PTGS_OK &&
        (hipMemcpyAsync(h.data(), hits, h.size() * sizeof(ptgs_hitdata), hipMemcpyDeviceToHost, s) != hipSuccess ||
         hipStreamSynchronize(s) != hipSuccess))
      rc = PTGS_EHIP;
    ptgs_device_free(ctx, hits);
    if (rc) return rc;
    if ((rc = ptgs_write_ply((root + "/points3d.ply").c_str(), h.data(), d->num_samples, &npoints))) return rc;
  }
  if (d->capture_images) {
    auto write = [&](const char* name, const std::vector<std::string>& p, const std::vector<float>& T) {
      std::vector<const char*> cp;
      for (const std::string& x : p) cp.push_back(x.c_str());
      return ptgs_write_transforms_json((root + "/" + name).c_str(), d->fov_deg, aspect, (uint32_t)p.size(),
                                        cp.data(), T.data());
    };
    if ((rc = write("transforms_train.json", paths_train, transforms_train))) return rc;
    if ((rc = write("transforms_test.json", paths_test, transforms_test))) return rc;
  }
  return PTGS_OK;
}

}  // extern "C"
