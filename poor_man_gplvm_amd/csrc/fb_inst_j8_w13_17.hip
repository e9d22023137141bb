// Scan kernel instances: 8 latent(s) per lane, band half-widths 13, 17
// (see fb_kernels.h; split so that `make -j` compiles them in parallel).
#include "fb_kernels.h"

namespace pmg {
PMG_FB_INST(8, 13)
PMG_FB_INST(8, 17)
}  // namespace pmg
