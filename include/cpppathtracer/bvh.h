// bvh.h — SceneBVH of the drop-in API (reference include/bvh.h:8-39, cuSrc/bvh.cu).
//
// Same process-global semantics as the reference: AddObject registers object pointers
// (nullptr and duplicates ignored, bvh.cu:22-29); BuildBVH snapshots every object BY VALUE
// (bvh.cu:43) into a median-split BVH and returns a handle; UpdateObject re-copies one object
// and refits its ancestors (bvh.cu:144-157); ReleaseBVH forgets everything.  The device-side
// TraceRay is the HIP traversal kernel.
#pragma once

#include <vector>

#include "object.h"

class SceneBVH;
typedef SceneBVH* SceneBVHGPUHandle;

class SceneBVH {
public:
    static void AddObject(Object* obj);
    static SceneBVHGPUHandle BuildBVH();
    static void UpdateObject(Object* obj);
    static void ReleaseBVH();

    // Build-time snapshot shared with PathTracer (by-value copies in AddObject order).
    static const std::vector<cpt_object>& Snapshot();
    // Bumped by BuildBVH (and ReleaseBVH); renderers rebuild when it changes.
    static uint64_t BuildId();
    // Snapshot indices UpdateObject touched since the last BuildBVH, in call order;
    // renderers refit them (cpt_update_object) instead of rebuilding, like bvh.cu:144-157.
    static std::vector<int> UpdateLog();
    // Index of `obj` in the snapshot (-1 if unknown).
    static int IndexOf(const Object* obj);
};
