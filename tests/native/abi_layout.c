/* Compile-time check of include/ptgs/ptgs.h's struct layouts from plain C11 (tests/test_abi.py compiles
 * this with gcc and g++): the header's PTGS_LAYOUT_ASSERTs hold every size / offset of the reference's
 * Helpers/GeneralHeaders.h structs, so this file fails to compile on any drift.
 * The checks below add the layouts that only the library's own entry points define. */
#include <stddef.h>

#include "ptgs/ptgs.h"

PTGS_LAYOUT_ASSERT(sizeof(ptgs_texture) == 24, "ptgs_texture is 24 B");
PTGS_LAYOUT_ASSERT(offsetof(ptgs_texture, srgb) == 16, "ptgs_texture.srgb at 16");
PTGS_LAYOUT_ASSERT(offsetof(ptgs_scene_desc, textures) == offsetof(ptgs_scene_desc, blue_noise_size) + 8,
                   "ptgs_scene_desc.textures after blue_noise_size");
PTGS_LAYOUT_ASSERT(offsetof(ptgs_scene_desc, num_textures) == offsetof(ptgs_scene_desc, textures) + 8,
                   "ptgs_scene_desc.num_textures after textures");
PTGS_LAYOUT_ASSERT(sizeof(ptgs_splat_status) == 80, "ptgs_splat_status is 80 B (ABI 3)");
PTGS_LAYOUT_ASSERT(offsetof(ptgs_splat_status, spilled_tiles) == 56, "ptgs_splat_status.spilled_tiles at 56");
PTGS_LAYOUT_ASSERT(offsetof(ptgs_splat_status, spill_demand) == 76, "ptgs_splat_status.spill_demand at 76");
PTGS_LAYOUT_ASSERT(sizeof(ptgs_splat_stats) == 20, "ptgs_splat_stats is 20 B");

int ptgs_abi_layout_checked(void) { return PTGS_ABI_VERSION; }
