// cpt_api.cpp — the reference-shaped C++ construction API (include/cpppathtracer/*.h) on top
// of the C-ABI (include/cpt.h).  Host code only; every GPU operation goes through cpt_*.
#include <dlfcn.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <algorithm>
#include <map>
#include <mutex>
#include <set>
#include <sstream>

#include "../../include/cpppathtracer/path_tracer.h"

// ======================================================================================
// Object (object.cu:134-170)
// ======================================================================================
float3 Object::GetAABBMax() {
    float3 m = make_float3(0.f);
    const float tol = BOUNCE_RAY_TMIN * 5.f;
    switch (type_) {
        case PrimitiveType::Sphere: m = center_ + make_float3(ABS(radius_)); break;
        case PrimitiveType::Platform: m = make_float3(DEFAULT_RAY_TMAX * 5, y_pos_ + tol, DEFAULT_RAY_TMAX * 5); break;
        case PrimitiveType::Cylinder:
            m = make_float3(center_.x + ABS(radius_), center_.y + height_ / 2 + tol, center_.z + ABS(radius_));
            break;
        default: break;
    }
    return m;
}

float3 Object::GetAABBMin() {
    float3 m = make_float3(0.f);
    const float tol = BOUNCE_RAY_TMIN * 5.f;
    switch (type_) {
        case PrimitiveType::Sphere: m = center_ - make_float3(ABS(radius_)); break;
        case PrimitiveType::Platform: m = make_float3(-DEFAULT_RAY_TMAX * 5, y_pos_ - tol, -DEFAULT_RAY_TMAX * 5); break;
        case PrimitiveType::Cylinder:
            m = make_float3(center_.x - ABS(radius_), center_.y - height_ / 2 - tol, center_.z - ABS(radius_));
            break;
        default: break;
    }
    return m;
}

// ======================================================================================
// MotionalCamera (motional_camera.cu)
// ======================================================================================
static std::mutex camera_mutex;   // motional_camera.cu:12

MotionalCamera::MotionalCamera()
    : width_(1920), height_(1080), cur_sample_idx_(0), origin_(make_float3(0.f)), look_at_(make_float3(0.f, 0.f, 1.f)) {}
MotionalCamera::MotionalCamera(int width, int height)
    : width_(width), height_(height), cur_sample_idx_(0), origin_(make_float3(0.f)), look_at_(make_float3(0.f, 0.f, 1.f)) {}
MotionalCamera::MotionalCamera(int width, int height, float3 ori, float3 at)
    : width_(width), height_(height), cur_sample_idx_(0), origin_(ori), look_at_(at) {}
MotionalCamera::~MotionalCamera() {}

void MotionalCamera::Refresh() { cur_sample_idx_ = 0; }
void MotionalCamera::SetViewFov(float fov) { view_fov_ = fov; }
void MotionalCamera::Resize(int width, int height) { width_ = width; height_ = height; }
void MotionalCamera::SetOrigin(float3 ori) { origin_ = ori; }
void MotionalCamera::SetOrigin(float x, float y, float z) { origin_ = make_float3(x, y, z); }
void MotionalCamera::SetLookAt(float3 look_at) { look_at_ = look_at; }
void MotionalCamera::SetLookAt(float x, float y, float z) { look_at_ = make_float3(x, y, z); }

// Interactive camera controls (motional_camera.cu:76-168).  SURVEY.md §2 puts them outside
// the hot path; they are kept only so the public MotionalCamera API is complete.  This is an
// API-behaviour restatement: a move is origin/look_at += (k * move_speed) * axis along the
// eye's left / back / up axis (a negated axis for the opposite move, which rounds exactly as
// the reference's -=), and a turn re-normalises look_at onto the unit sphere around the eye,
// steps it along the eye's left or up axis and re-normalises, with the reference's float
// operations in the reference's order.
namespace {
float3 eye_left(const MotionalCamera& c) { return -normalize(cross(c.vup, normalize(c.origin_ - c.look_at_))); }
float3 eye_back(const MotionalCamera& c) { return -normalize(cross(eye_left(c), c.vup)); }

void translate(MotionalCamera& c, float3 axis, float k) {
    c.origin_ += k * c.move_speed_ * axis;
    c.look_at_ += k * c.move_speed_ * axis;
}

// `up`: step along the up axis (else the left axis) by d.
void turn(MotionalCamera& c, bool up, float d) {
    c.look_at_ = c.origin_ + normalize(c.look_at_ - c.origin_);
    const float3 w = normalize(c.look_at_ - c.origin_);
    const float3 left = normalize(cross(c.vup, w));
    const float3 axis = up ? normalize(cross(w, left)) : left;
    c.look_at_ += d * axis;
    c.look_at_ = c.origin_ + normalize(c.look_at_ - c.origin_);
}
}  // namespace

void MotionalCamera::MoveEyeLeft(float k) { translate(*this, eye_left(*this), k); }
void MotionalCamera::MoveEyeRight(float k) { translate(*this, -eye_left(*this), k); }
void MotionalCamera::MoveEyeForward(float k) { translate(*this, -eye_back(*this), k); }
void MotionalCamera::MoveEyeBackward(float k) { translate(*this, eye_back(*this), k); }
void MotionalCamera::MoveEyeUp(float k) { translate(*this, vup, k); }
void MotionalCamera::MoveEyeDown(float k) { translate(*this, -vup, k); }
void MotionalCamera::RotateAroundUp(float dy) { turn(*this, true, dy); }
void MotionalCamera::RotateAroundDown(float dy) { turn(*this, true, -dy); }
void MotionalCamera::RotateAroundLeft(float dx) { turn(*this, false, dx); }
void MotionalCamera::RotateAroundRight(float dx) { turn(*this, false, -dx); }
void MotionalCamera::ScaleFov(float d) { view_fov_ = (float)(view_fov_ + d * M_PI / 180.0f); }
void MotionalCamera::Lock() { camera_mutex.lock(); }
void MotionalCamera::Unlock() { camera_mutex.unlock(); }

MotionalCamera MotionalCamera::GetCopy() {
    std::lock_guard<std::mutex> lock(camera_mutex);
    cpt_camera_get_copy(reinterpret_cast<cpt_camera*>(this));   // basis + cur_sample_idx_++
    return *this;
}

// ======================================================================================
// SceneBVH statics (bvh.cu:16-29, 116-165)
// ======================================================================================
namespace {
std::mutex bvh_mutex;
std::vector<Object*> bvh_objs;
std::set<Object*> bvh_seen;
std::vector<cpt_object> bvh_built;      // BuildBVH's by-value copies (bvh.cu:43)
std::vector<cpt_object> bvh_current;    // ... with UpdateObject's re-copies
std::vector<uint64_t> bvh_updates;      // UpdateObject calls per object since the build
uint64_t bvh_build_id = 0, bvh_revision = 0;
SceneBVH* const bvh_handle = reinterpret_cast<SceneBVH*>(&bvh_built);   // opaque, non-null

// texture registry
std::mutex tex_mutex;
std::map<PocaTexture, PocaTextureData> tex_registry;
PocaTexture tex_next = 1;
}  // namespace

void SceneBVH::AddObject(Object* obj) {
    std::lock_guard<std::mutex> lk(bvh_mutex);
    if (obj == nullptr || bvh_seen.count(obj)) return;
    bvh_objs.push_back(obj);
    bvh_seen.insert(obj);
}

SceneBVHGPUHandle SceneBVH::BuildBVH() {
    std::lock_guard<std::mutex> lk(bvh_mutex);
    bvh_built.resize(bvh_objs.size());
    for (size_t i = 0; i < bvh_objs.size(); ++i) std::memcpy(&bvh_built[i], bvh_objs[i], sizeof(cpt_object));
    bvh_current = bvh_built;
    bvh_updates.assign(bvh_built.size(), 0);
    bvh_build_id++;
    bvh_revision++;
    return bvh_handle;
}

void SceneBVH::UpdateObject(Object* obj) {
    std::lock_guard<std::mutex> lk(bvh_mutex);
    for (size_t i = 0; i < bvh_objs.size() && i < bvh_current.size(); ++i)
        if (bvh_objs[i] == obj) {
            std::memcpy(&bvh_current[i], obj, sizeof(cpt_object));
            bvh_updates[i]++;
            bvh_revision++;
            return;
        }
}

void SceneBVH::ReleaseBVH() {
    std::lock_guard<std::mutex> lk(bvh_mutex);
    bvh_objs.clear();
    bvh_seen.clear();
    bvh_built.clear();
    bvh_current.clear();
    bvh_updates.clear();
    bvh_build_id++;
    bvh_revision++;
}

uint64_t SceneBVH::BuildId() {
    std::lock_guard<std::mutex> lk(bvh_mutex);
    return bvh_build_id;
}

uint64_t SceneBVH::Revision() {
    std::lock_guard<std::mutex> lk(bvh_mutex);
    return bvh_revision;
}

void SceneBVH::GetState(uint64_t& build_id, uint64_t& revision, std::vector<cpt_object>* built,
                        std::vector<cpt_object>& current, std::vector<uint64_t>& updates) {
    std::lock_guard<std::mutex> lk(bvh_mutex);
    build_id = bvh_build_id;
    revision = bvh_revision;
    if (built) *built = bvh_built;
    current = bvh_current;
    updates = bvh_updates;
}

int SceneBVH::IndexOf(const Object* obj) {
    std::lock_guard<std::mutex> lk(bvh_mutex);
    for (size_t i = 0; i < bvh_objs.size(); ++i)
        if (bvh_objs[i] == obj) return (int)i;
    return -1;
}

// ======================================================================================
// PocaTextureUtils (textures.cu:14-66)
// ======================================================================================
static bool load_cptex(const std::string& path, PocaTextureData& t) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    char magic[8];
    uint32_t hdr[4];
    if (!f.read(magic, 8) || std::memcmp(magic, "CPTTEX01", 8) != 0) return false;
    if (!f.read(reinterpret_cast<char*>(hdr), sizeof(hdr))) return false;
    t.width = (int)hdr[0];
    t.height = (int)hdr[1];
    t.valid_cols = (int)hdr[2];
    t.rgba.resize((size_t)t.valid_cols * t.height * 4);
    return (bool)f.read(reinterpret_cast<char*>(t.rgba.data()), (std::streamsize)t.rgba.size());
}

static bool load_ppm(const std::string& path, PocaTextureData& t) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::string magic;
    f >> magic;
    if (magic != "P6") return false;
    int w = 0, h = 0, maxv = 0;
    f >> w >> h >> maxv;
    f.get();
    if (w <= 0 || h <= 0 || maxv != 255) return false;
    std::vector<uint8_t> rgb((size_t)w * h * 3);
    if (!f.read(reinterpret_cast<char*>(rgb.data()), (std::streamsize)rgb.size())) return false;
    // textures.cu:32-33: cudaMemcpy2DToArray copies `width` BYTES per row = width/4 texels.
    t.width = w;
    t.height = h;
    t.valid_cols = w / 4;
    t.rgba.resize((size_t)t.valid_cols * h * 4);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < t.valid_cols; ++x) {
            const uint8_t* s = &rgb[((size_t)y * w + x) * 3];
            uint8_t* d = &t.rgba[((size_t)y * t.valid_cols + x) * 4];
            d[0] = s[0]; d[1] = s[1]; d[2] = s[2]; d[3] = 255;
        }
    return true;
}

static int address_mode_of(PocaAddressMode m) {
    switch (m) {
        case PocaAddressMode::Wrap: return CPT_ADDRESS_WRAP;
        case PocaAddressMode::Clamp: return CPT_ADDRESS_CLAMP;
        case PocaAddressMode::Border: return CPT_ADDRESS_BORDER;
        default: return CPT_ADDRESS_MIRROR;
    }
}

PocaTexture PocaTextureUtils::AddTexByFile(std::string file_path, PocaAddressMode addr_mode, PocaFilterMode filter_mode) {
    PocaTextureData t;
    t.addr = addr_mode;
    t.filter = filter_mode;
    if (!load_cptex(file_path, t) && !load_ppm(file_path, t)) {
        fprintf(stderr, "[cpt] AddTexByFile: cannot load %s (.cptex or binary PPM)\n", file_path.c_str());
        return 0;
    }
    std::lock_guard<std::mutex> lk(tex_mutex);
    PocaTexture h = tex_next++;
    tex_registry[h] = std::move(t);
    return h;
}

void PocaTextureUtils::DestroyTexture(PocaTexture tex) {
    std::lock_guard<std::mutex> lk(tex_mutex);
    tex_registry.erase(tex);
}

const PocaTextureData* PocaTextureUtils::Get(PocaTexture tex) {
    std::lock_guard<std::mutex> lk(tex_mutex);
    auto it = tex_registry.find(tex);
    return it == tex_registry.end() ? nullptr : &it->second;
}

// ======================================================================================
// PathTracer (path_tracer.cu:29-319)
// ======================================================================================
static std::string default_sky_path() {
    if (const char* e = getenv("CPT_SKY_PATH")) return e;
    {
        std::ifstream f("assets/sky.cptex");
        if (f) return "assets/sky.cptex";
    }
    Dl_info info;
    if (dladdr(reinterpret_cast<void*>(&default_sky_path), &info) && info.dli_fname) {
        std::string so = info.dli_fname;
        std::string dir = so.substr(0, so.find_last_of('/'));
        return dir + "/../assets/sky.cptex";
    }
    return "assets/sky.cptex";
}

PathTracer::PathTracer() {}

PathTracer::~PathTracer() {
    Stop();
    if (output_pinned_) (void)cpt_host_unregister(output_buffer_.data());
    for (Tile& t : tiles_)
        if (t.ctx) cpt_destroy(t.ctx);
    if (frame_) cpt_destroy(frame_);
}

bool PathTracer::Fail(const char* what, cpt_ctx* ctx) {
    if (!ctx) ctx = FrameCtx();
    err_ = std::string(what) + ": " + (ctx ? cpt_last_error(ctx) : cpt_last_error(nullptr));
    fprintf(stderr, "[cpt] %s\n", err_.c_str());   // the reference logs and continues
    return false;
}

void PathTracer::AddObject(Object* obj) { SceneBVH::AddObject(obj); }

void PathTracer::SetCamera(std::shared_ptr<MotionalCamera>& camera) { camera_ = camera; }
std::shared_ptr<MotionalCamera> PathTracer::GetCamera() { return camera_; }

bool PathTracer::SetMaxRecursionDepth(uint depth) {
    if (depth > MAX_RECURSION_DEPTH_SET) {
        err_ = "SetMaxRecursionDepth: depth must be <= 32";
        return false;
    }
    max_recursion_depth_ = depth;
    return true;
}

void PathTracer::SetSeed(uint64_t seed) {
    std::lock_guard<std::mutex> lk(mu_);
    seed_ = seed;
    for (Tile& t : tiles_) t.rng_ready = false;
}

bool PathTracer::SetDevice(int device) {
    std::lock_guard<std::mutex> lk(mu_);
    if (!tiles_.empty()) {
        err_ = "SetDevice: the context already exists";
        return false;
    }
    device_ = device;
    device_list_.clear();
    return true;
}

bool PathTracer::SetDevices(int n) {
    if (n < 1) {
        err_ = "SetDevices: n must be >= 1";
        return false;
    }
    int visible = 0;
    if (cpt_get_device_count(&visible) != CPT_OK || visible < 1) {
        err_ = "SetDevices: no HIP device visible";
        return false;
    }
    std::vector<int> devs(n);
    for (int i = 0; i < n; ++i) devs[i] = i % visible;
    return SetDevices(devs);
}

bool PathTracer::SetDevices(const std::vector<int>& devices) {
    std::lock_guard<std::mutex> lk(mu_);
    if (!tiles_.empty()) {
        err_ = "SetDevices: the contexts already exist";
        return false;
    }
    if (devices.empty()) {
        err_ = "SetDevices: empty device list";
        return false;
    }
    device_list_ = devices.size() > 1 ? devices : std::vector<int>{};
    device_ = devices[0];
    return true;
}

bool PathTracer::SetEnvTexture(PocaTexture tex) {
    std::lock_guard<std::mutex> lk(mu_);
    env_ = tex;
    for (Tile& t : tiles_) t.env_uploaded = false;
    return true;
}

// One context per device of the row tiling (a single one without SetDevices), plus, with
// several, the frame context on the first device that receives the gathered tiles.
bool PathTracer::EnsureContext() {
    if (!tiles_.empty()) return true;
    const std::vector<int> devs = device_list_.empty() ? std::vector<int>{device_} : device_list_;
    std::vector<Tile> tiles(devs.size());
    for (size_t i = 0; i < devs.size(); ++i) {
        tiles[i].device = devs[i];
        if (cpt_create(devs[i], &tiles[i].ctx) != CPT_OK) {
            tiles[i].ctx = nullptr;
            for (Tile& t : tiles)
                if (t.ctx) cpt_destroy(t.ctx);
            return Fail("cpt_create", nullptr);
        }
    }
    if (devs.size() > 1 && cpt_create(devs[0], &frame_) != CPT_OK) {
        frame_ = nullptr;
        for (Tile& t : tiles) cpt_destroy(t.ctx);
        return Fail("cpt_create", nullptr);
    }
    tiles_ = std::move(tiles);
    return true;
}

// Binds every material texture handle `objs` use that the context does not hold yet.
bool PathTracer::BindTextures(Tile& tile, const std::vector<cpt_object>& objs) {
    for (const cpt_object& o : objs) {
        if (!o.material.have_tex) continue;
        const uint64_t h = o.material.u.tex;
        if (std::find(tile.bound_textures.begin(), tile.bound_textures.end(), h) != tile.bound_textures.end()) continue;
        const PocaTextureData* t = PocaTextureUtils::Get(h);
        if (!t) { err_ = "textured material uses an unknown PocaTexture handle"; return false; }
        if (cpt_bind_texture(tile.ctx, h, t->rgba.data(), t->width, t->height, t->valid_cols, address_mode_of(t->addr),
                             t->filter == PocaFilterMode::Point ? CPT_FILTER_POINT : CPT_FILTER_LINEAR) != CPT_OK)
            return Fail("cpt_bind_texture", tile.ctx);
        tile.bound_textures.push_back(h);
    }
    return true;
}

// Brings one context to a snapshot of SceneBVH's state: a new build is uploaded as BuildBVH
// copied it (the reference's topology), then the objects UpdateObject re-copied since are refit
// in one batch (bvh.cu:144-157).
bool PathTracer::SyncTile(Tile& tile, const SceneSnap& snap) {
    if (!tile.scene_synced || snap.rev != tile.scene_rev) {
        if (!tile.scene_synced || snap.build != tile.scene_build) {
            tile.bound_textures.clear();
            if (!BindTextures(tile, snap.built)) return false;
            if (cpt_set_scene(tile.ctx, snap.built.empty() ? nullptr : snap.built.data(), (int)snap.built.size()) != CPT_OK)
                return Fail("cpt_set_scene", tile.ctx);
            tile.scene_build = snap.build;
            tile.updates_seen.assign(snap.built.size(), 0);
        }
        std::vector<int> idx;
        std::vector<cpt_object> objs;
        for (size_t i = 0; i < snap.updates.size() && i < tile.updates_seen.size(); ++i)
            if (snap.updates[i] != tile.updates_seen[i]) {
                idx.push_back((int)i);
                objs.push_back(snap.current[i]);
            }
        if (!idx.empty()) {
            if (!BindTextures(tile, objs)) return false;
            if (cpt_update_objects(tile.ctx, (int)idx.size(), idx.data(), objs.data()) != CPT_OK)
                return Fail("cpt_update_objects", tile.ctx);
        }
        tile.updates_seen = snap.updates;
        tile.scene_rev = snap.rev;
        tile.scene_synced = true;
    }
    if (!tile.env_uploaded) {
        if (env_ == 0) env_ = PocaTextureUtils::AddTexByFile(default_sky_path());   // path_tracer.cu:47
        const PocaTextureData* t = PocaTextureUtils::Get(env_);
        int rc = t ? cpt_set_env_texture(tile.ctx, t->rgba.data(), t->width, t->height, t->valid_cols)
                   : cpt_set_env_texture(tile.ctx, nullptr, 1, 1, 0);
        if (rc != CPT_OK) return Fail("cpt_set_env_texture", tile.ctx);
        tile.env_uploaded = true;
    }
    return true;
}

// One snapshot for the whole pass: an UpdateObject from another thread lands either before
// every tile or after all of them, never between two tiles of one frame.
bool PathTracer::SyncScene() {
    if (!EnsureContext()) return false;
    SceneSnap snap;
    bool need = false;
    const uint64_t rev = SceneBVH::Revision();
    for (const Tile& t : tiles_) need = need || !t.scene_synced || t.scene_rev != rev;
    if (need) {
        SceneBVH::GetState(snap.build, snap.rev, &snap.built, snap.current, snap.updates);
    } else {
        snap.build = tiles_[0].scene_build;
        snap.rev = tiles_[0].scene_rev;
    }
    for (Tile& t : tiles_)
        if (!SyncTile(t, snap)) return false;
    return true;
}

// Image rows of tile r of n: interleaved 8-row blocks (cpppathtracer_amd/tiling.py).
static std::vector<int32_t> tile_rows(int height, int n, int r) {
    std::vector<int32_t> rows;
    for (int y = 0; y < height; ++y)
        if ((y / 8) % n == r) rows.push_back(y);
    return rows;
}

// InitBuffers (path_tracer.cu:44-115): per-pixel buffers and RNG when the size changes.
bool PathTracer::EnsureFrame(const MotionalCamera& cam) {
    const int n = (int)tiles_.size();
    if (cam.width_ != width_ || cam.height_ != height_) {
        for (int r = 0; r < n; ++r) {
            const std::vector<int32_t> rows = tile_rows(cam.height_, n, r);
            const int rc = n == 1 ? cpt_set_frame(tiles_[r].ctx, cam.width_, cam.height_, nullptr, 0)
                                  : cpt_set_frame(tiles_[r].ctx, cam.width_, cam.height_, rows.data(), (int)rows.size());
            if (rc != CPT_OK) return Fail("cpt_set_frame", tiles_[r].ctx);
            tiles_[r].rng_ready = false;
        }
        if (frame_ && cpt_set_frame(frame_, cam.width_, cam.height_, nullptr, 0) != CPT_OK) return Fail("cpt_set_frame", frame_);
        width_ = cam.width_;
        height_ = cam.height_;
        if (output_pinned_) (void)cpt_host_unregister(output_buffer_.data());
        output_buffer_.assign((size_t)width_ * height_ * 4, 0);
        // pinned, so each pass's frame reaches it without a staging copy (cpt_denoise_mix); a
        // buffer that cannot be pinned still works through the copy
        output_pinned_ = !output_buffer_.empty() &&
                         cpt_host_register(output_buffer_.data(), output_buffer_.size()) == CPT_OK;
    }
    for (Tile& t : tiles_)
        if (!t.rng_ready) {
            if (cpt_init_rng(t.ctx, seed_) != CPT_OK) return Fail("cpt_init_rng", t.ctx);
            t.rng_ready = true;
        }
    return true;
}

// One render of `spp` passes: every tile's launch is queued first (each context's work runs on
// its own device and stream), then the tiles are gathered into the frame context.
bool PathTracer::RenderPass(MotionalCamera& cam, int spp, bool accumulate) {
    if (!SyncScene() || !EnsureFrame(cam)) return false;
    // many passes per pixel: heaviest tiles first (same image, shorter tail)
    // few passes (the DispatchRay loop): heaviest tiles first by the previous pass's work, no pilot
    const uint32_t flags = CPT_RENDER_AUX | (accumulate ? CPT_RENDER_ACCUMULATE : 0u) |
                           (ordered_walk_ ? CPT_TRAVERSAL_ORDERED : 0u) |
                           (spp >= 64 ? CPT_SCHEDULE_COST : CPT_SCHEDULE_PREVIOUS);
    if (!frame_) {
        if (cpt_render(tiles_[0].ctx, reinterpret_cast<const cpt_camera*>(&cam), spp, (int)max_recursion_depth_,
                       flags | CPT_RENDER_SYNC) != CPT_OK)
            return Fail("cpt_render", tiles_[0].ctx);
        return true;
    }
    for (Tile& t : tiles_)
        if (cpt_render(t.ctx, reinterpret_cast<const cpt_camera*>(&cam), spp, (int)max_recursion_depth_, flags) != CPT_OK)
            return Fail("cpt_render", t.ctx);
    // every gather queues behind its tile's render (events, no host wait); one wait at the end
    for (Tile& t : tiles_)
        if (cpt_gather_rows(frame_, t.ctx) != CPT_OK) return Fail("cpt_gather_rows", frame_);
    if (cpt_synchronize(frame_) != CPT_OK) return Fail("cpt_synchronize", frame_);
    for (Tile& t : tiles_)   // the tiles' device errors (their work is done by now)
        if (cpt_synchronize(t.ctx) != CPT_OK) return Fail("cpt_synchronize", t.ctx);
    return true;
}

void PathTracer::InitPipeline() {
    SceneBVH::BuildBVH();   // bvh.cu:116-120
    if (running_.exchange(true)) return;
    worker_ = std::thread(&PathTracer::PipelineLoop, this);
}

void PathTracer::DispatchRay(DispatchRayArgs args) {
    {
        std::lock_guard<std::mutex> lk(mu_);
        tasks_queue_.push_back(args);
    }
    cv_.notify_one();
}

// PipelineLoop (path_tracer.cu:256-306): one sample per pixel per task, then denoise + mix and
// the callback with the BGRA8 frame, on this thread.
void PathTracer::PipelineLoop() {
    if (camera_) {
        MotionalCamera first = camera_->GetCopy();   // the reference's InitBuffers(GetCopy()) (:258)
        std::lock_guard<std::mutex> lk(mu_);
        if (SyncScene()) EnsureFrame(first);
    }
    while (running_.load()) {
        DispatchRayArgs task;
        {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return !tasks_queue_.empty() || !running_.load(); });
            if (!running_.load()) break;
            task = tasks_queue_.front();
            tasks_queue_.pop_front();
        }
        if (!camera_) continue;
        MotionalCamera cma = camera_->GetCopy();
        bool ok;
        {
            std::lock_guard<std::mutex> lk(mu_);
            ok = RenderPass(cma, 1, false);
            if (ok && cpt_denoise_mix(FrameCtx(), cma.cur_sample_idx_, output_buffer_.data()) != CPT_OK)
                ok = Fail("cpt_denoise_mix");
        }
        if (ok && task.Callback) task.Callback(output_buffer_.data(), width_, height_, task.cbParam);
    }
}

void PathTracer::Stop() {
    if (!running_.exchange(false)) return;
    cv_.notify_all();
    if (worker_.joinable()) worker_.join();
}

bool PathTracer::Render(int spp, bool accumulate) {
    if (!camera_) {
        err_ = "Render: SetCamera first";
        return false;
    }
    if (SceneBVH::BuildId() == 0) SceneBVH::BuildBVH();
    MotionalCamera cma = camera_->GetCopy();
    std::lock_guard<std::mutex> lk(mu_);
    return RenderPass(cma, spp, accumulate);
}

bool PathTracer::ReadRadiance(std::vector<float>& rgb) {
    std::lock_guard<std::mutex> lk(mu_);
    if (!FrameCtx() || width_ == 0) {
        err_ = "ReadRadiance: nothing rendered";
        return false;
    }
    std::vector<float> acc((size_t)width_ * height_ * 4);
    if (cpt_read_accum(FrameCtx(), acc.data()) != CPT_OK) return Fail("cpt_read_accum");
    rgb.resize((size_t)width_ * height_ * 3);
    for (size_t i = 0; i < (size_t)width_ * height_; ++i) {
        float n = acc[4 * i + 3] > 0.f ? acc[4 * i + 3] : 1.f;
        rgb[3 * i] = acc[4 * i] / n;
        rgb[3 * i + 1] = acc[4 * i + 1] / n;
        rgb[3 * i + 2] = acc[4 * i + 2] / n;
    }
    return true;
}

bool PathTracer::ReadFrameBGRA(std::vector<uint8_t>& bgra) {
    std::lock_guard<std::mutex> lk(mu_);
    bgra = output_buffer_;
    return !bgra.empty();
}

bool PathTracer::SaveRadiancePFM(const std::string& path) {
    std::vector<float> rgb;
    if (!ReadRadiance(rgb)) return false;
    std::ofstream f(path, std::ios::binary);
    if (!f) {
        err_ = "SaveRadiancePFM: cannot open " + path;
        return false;
    }
    f << "PF\n" << width_ << " " << height_ << "\n-1.0\n";
    for (int y = height_ - 1; y >= 0; --y)   // PFM rows are bottom-to-top
        f.write(reinterpret_cast<const char*>(&rgb[(size_t)y * width_ * 3]), (std::streamsize)width_ * 3 * sizeof(float));
    return (bool)f;
}

// Counters summed over the tiles (the render flags do not ask for CPT_RENDER_STATS, so these
// are the counters of the last counting render; GetStats after cpt-level counting renders).
bool PathTracer::GetStats(cpt_stats* out) {
    std::lock_guard<std::mutex> lk(mu_);
    if (tiles_.empty() || !out) return false;
    *out = cpt_stats{};
    for (Tile& t : tiles_) {
        cpt_stats s{};
        if (cpt_get_stats(t.ctx, &s) != CPT_OK) return Fail("cpt_get_stats", t.ctx);
        out->segments += s.segments;
        out->node_visits += s.node_visits;
        out->prim_tests += s.prim_tests;
        out->hits += s.hits;
        out->misses += s.misses;
    }
    return true;
}
