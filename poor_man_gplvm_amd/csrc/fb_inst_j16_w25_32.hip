// Scan kernel instances: 16 latent(s) per lane, band half-widths 25, 32
// (see fb_kernels.h; split so that `make -j` compiles them in parallel).
#include "fb_kernels.h"

namespace pmg {
PMG_FB_INST(16, 25)
PMG_FB_INST(16, 32)
}  // namespace pmg
