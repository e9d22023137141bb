// Scan kernel instances: 2 latent(s) per lane, band half-widths 5, 9, 13, 17, 25, 32
// (see fb_kernels.h; split so that `make -j` compiles them in parallel).
#include "fb_kernels.h"

namespace pmg {
PMG_FB_INST(2, 5)
PMG_FB_INST(2, 9)
PMG_FB_INST(2, 13)
PMG_FB_INST(2, 17)
PMG_FB_INST(2, 25)
PMG_FB_INST(2, 32)
}  // namespace pmg
