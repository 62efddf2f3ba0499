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

    // ---- additions: the state a renderer uploads ---------------------------------------
    // Bumped by BuildBVH (and ReleaseBVH); renderers rebuild when it changes.
    static uint64_t BuildId();
    // Bumped by every BuildBVH / UpdateObject / ReleaseBVH: a renderer whose copy is at this
    // revision has nothing to do.
    static uint64_t Revision();
    // One consistent copy, taken under one lock: the build id and revision, the objects as
    // BuildBVH copied them (`built`, the topology the reference builds; filled only when
    // non-null), their current values and a per-object count of UpdateObject calls since the
    // build.  A renderer refits the objects whose count moved (cpt_update_objects).
    static void GetState(uint64_t& build_id, uint64_t& revision, std::vector<cpt_object>* built,
                         std::vector<cpt_object>& current, std::vector<uint64_t>& updates);
    // Index of `obj` in the snapshot (-1 if unknown).
    static int IndexOf(const Object* obj);
};
