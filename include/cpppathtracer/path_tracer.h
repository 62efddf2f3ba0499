// path_tracer.h — PathTracer, the drop-in surface of the reference's hot path
// (reference include/path_tracer.h:15-50, cuSrc/path_tracer.cu).
//
// Reference interface, same names and meaning:
//   AddObject(Object*)            register an object (path_tracer.cu:29-34)
//   InitPipeline()                build the BVH, start the render thread (:308-314)
//   DispatchRay(DispatchRayArgs)  queue one pass; the render thread runs SamplePixel for one
//                                 sample per pixel, the 5x5 denoise and the running-mean Mix,
//                                 then calls Callback(BGRA8, width, height, cbParam) (:256-306)
//   SetCamera / GetCamera
// Additions the headless configs need (the reference has no setters for these):
//   SetMaxRecursionDepth, SetSeed, SetDevice, SetEnvTexture, Render(spp) (synchronous),
//   ReadRadiance, ReadFrameBGRA, SaveRadiancePFM, GetStats, Stop.
// Errors: the reference logs CUDA errors and continues; here every call that reaches the
// GPU returns false on failure and LastError() holds the message (no exceptions).
#pragma once

#include <atomic>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "bvh.h"
#include "motional_camera.h"
#include "object.h"
#include "ray_tracing_common.h"
#include "textures.h"

#define MAX_RECURSION_DEPTH_SET 32

class PathTracer {
public:
    PathTracer();
    ~PathTracer();

    void AddObject(Object* obj);
    void InitPipeline();
    void DispatchRay(DispatchRayArgs args);
    void SetCamera(std::shared_ptr<MotionalCamera>& camera);
    std::shared_ptr<MotionalCamera> GetCamera();

    // ---- additions ------------------------------------------------------------------
    bool SetMaxRecursionDepth(uint depth);      // 0..32; reference default 8 (path_tracer.h:43)
    void SetSeed(uint64_t seed);                // reference seeds with clock() (path_tracer.cu:107)
    bool SetDevice(int device);                 // before the first render
    bool SetEnvTexture(PocaTexture tex);        // default: textures/sky (assets/sky.cptex)
    // BVH walk: true (default) = CPT_TRAVERSAL_ORDERED (same image, fewer node visits);
    // false = the reference's right-first DFS order (its node/prim counts in GetStats).
    void SetOrderedTraversal(bool on) { ordered_walk_ = on; }
    // Synchronous `spp` passes into the radiance accumulator (accumulate=false restarts it).
    bool Render(int spp, bool accumulate = true);
    // Per-pixel mean radiance, rgb float[width*height*3] (row-major, y down).
    bool ReadRadiance(std::vector<float>& rgb);
    // Last display frame (denoised running mean), BGRA8[width*height*4].
    bool ReadFrameBGRA(std::vector<uint8_t>& bgra);
    bool SaveRadiancePFM(const std::string& path);
    bool GetStats(cpt_stats* out);
    void Stop();                                 // stop the render thread (also in ~PathTracer)
    const std::string& LastError() const { return err_; }

private:
    bool EnsureContext();
    bool SyncScene();
    bool BindTextures(const std::vector<cpt_object>& objs);
    bool EnsureFrame(const MotionalCamera& cam);
    bool RenderPass(MotionalCamera& cam, int spp, bool accumulate);
    void PipelineLoop();
    bool Fail(const char* what);

    cpt_ctx* ctx_ = nullptr;
    int device_ = 0;
    uint64_t seed_ = 1234;
    uint max_recursion_depth_ = 8;
    bool ordered_walk_ = true;
    int width_ = 0, height_ = 0;
    bool scene_synced_ = false;
    uint64_t scene_build_ = 0;      // SceneBVH::BuildId() uploaded to the context
    uint64_t scene_rev_ = 0;        // SceneBVH::Revision() the context is at
    std::vector<uint64_t> updates_seen_;       // per-object UpdateObject counts refit so far
    std::vector<uint64_t> bound_textures_;     // material texture handles bound on the context
    bool rng_ready_ = false;
    PocaTexture env_ = 0;
    bool env_uploaded_ = false;
    std::shared_ptr<MotionalCamera> camera_;
    std::vector<uint8_t> output_buffer_;   // BGRA8 handed to the callback
    std::string err_;

    std::mutex mu_;                        // guards the queue and the context
    std::condition_variable cv_;
    std::deque<DispatchRayArgs> tasks_queue_;
    std::atomic<bool> running_{false};
    std::thread worker_;
};
