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
//   SetMaxRecursionDepth, SetSeed, SetDevice, SetDevices (row tiling over several GPUs),
//   SetEnvTexture, Render(spp) (synchronous), ReadRadiance, ReadFrameBGRA, SaveRadiancePFM,
//   GetStats, Stop.
// Errors: the reference logs CUDA errors and continues; here every call that reaches the
// GPU returns false on failure and LastError() holds the message (no exceptions).
#pragma once

#include <algorithm>
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
    // Row tiling, before the first render: the image rows are dealt to n
    // contexts in interleaved 8-row blocks, one context per device (device i % visible devices,
    // or the listed devices; a device may repeat), each rendering its rows of every pass.  Each
    // pass's tiles are gathered into one frame on the first device (peer copies + a stitch
    // kernel, cpt_gather_rows), which ReadRadiance, ReadFrameBGRA and the DispatchRay display
    // path read.  A pixel's stream depends only on (seed, x, y): the image is bit-identical to
    // a single-device render.
    bool SetDevices(int n);
    bool SetDevices(const std::vector<int>& devices);
    int DeviceCount() const { return (int)std::max<size_t>(1, device_list_.size()); }
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
    // One libcpt context: the renderer of one row tile (or of the whole frame).
    struct Tile {
        cpt_ctx* ctx = nullptr;
        int device = 0;
        bool scene_synced = false;
        uint64_t scene_build = 0;      // SceneBVH::BuildId() uploaded to the context
        uint64_t scene_rev = 0;        // SceneBVH::Revision() the context is at
        std::vector<uint64_t> updates_seen;     // per-object UpdateObject counts refit so far
        std::vector<uint64_t> bound_textures;   // material texture handles bound on the context
        bool env_uploaded = false;
        bool rng_ready = false;
    };
    // One read of SceneBVH's state (SceneBVH::GetState), applied to every tile of a pass, so all
    // row tiles of a frame render the same scene revision.
    struct SceneSnap {
        uint64_t build = 0, rev = 0;
        std::vector<cpt_object> built, current;
        std::vector<uint64_t> updates;
    };
    bool EnsureContext();
    bool SyncScene();
    bool SyncTile(Tile& t, const SceneSnap& snap);
    bool BindTextures(Tile& t, const std::vector<cpt_object>& objs);
    bool EnsureFrame(const MotionalCamera& cam);
    bool RenderPass(MotionalCamera& cam, int spp, bool accumulate);
    void PipelineLoop();
    bool Fail(const char* what, cpt_ctx* ctx = nullptr);
    cpt_ctx* FrameCtx() const { return frame_ ? frame_ : (tiles_.empty() ? nullptr : tiles_[0].ctx); }

    std::vector<Tile> tiles_;       // one per device of the row tiling (one: the whole frame)
    cpt_ctx* frame_ = nullptr;      // row tiling: the gathered frame on the first device
    int device_ = 0;
    std::vector<int> device_list_;  // SetDevices (empty: the single device_)
    uint64_t seed_ = 1234;
    uint max_recursion_depth_ = 8;
    bool ordered_walk_ = true;
    int width_ = 0, height_ = 0;
    PocaTexture env_ = 0;
    std::shared_ptr<MotionalCamera> camera_;
    std::vector<uint8_t> output_buffer_;   // BGRA8 handed to the callback
    bool output_pinned_ = false;           // output_buffer_ registered with cpt_host_register
    std::string err_;

    std::mutex mu_;                        // guards the queue and the context
    std::condition_variable cv_;
    std::deque<DispatchRayArgs> tasks_queue_;
    std::atomic<bool> running_{false};
    std::thread worker_;
};
