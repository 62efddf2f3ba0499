// textures.h — PocaTextureUtils of the drop-in API (reference include/textures.h:7-16).
//
// AddTexByFile loads a texture file on the host and returns an opaque handle.  The reference
// decodes PNG with OpenCV (textures.cu:15-17); this build reads the raw `.cptex` format
// (tools/make_sky_fixture.py) and binary PPM (P6), since no image codec ships here.  The
// reference's upload quirk (only width/4 texels per row reach the texture, textures.cu:32-33)
// is applied to full-width images.  The sky is always sampled mirror + linear (the
// reference's defaults); material textures honour the handle's address and filter modes.
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

typedef uint64_t PocaTexture;   // replaces cudaTextureObject_t; 0 = none

enum class PocaAddressMode { Mirror, Wrap, Clamp, Border };
enum class PocaFilterMode { Linear, Point };

struct PocaTextureData {       // host copy owned by the texture registry
    std::vector<uint8_t> rgba;  // valid_cols x height RGBA8
    int width = 0;              // logical width
    int height = 0;
    int valid_cols = 0;
    PocaAddressMode addr = PocaAddressMode::Mirror;
    PocaFilterMode filter = PocaFilterMode::Linear;
};

class PocaTextureUtils {
public:
    static PocaTexture AddTexByFile(std::string file_path, PocaAddressMode addr_mode = PocaAddressMode::Mirror,
                                    PocaFilterMode filter_mode = PocaFilterMode::Linear);
    static void DestroyTexture(PocaTexture tex);
    // Host access to a loaded texture (NULL if unknown).
    static const PocaTextureData* Get(PocaTexture tex);
};
