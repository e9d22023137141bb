// Scan kernel instances: 4 latent(s) per lane, band half-widths 5, 9, 13
// (see fb_kernels.h; split so that `make -j` compiles them in parallel).
#include "fb_kernels.h"

namespace pmg {
PMG_FB_INST(4, 5)
PMG_FB_INST(4, 9)
PMG_FB_INST(4, 13)
}  // namespace pmg
