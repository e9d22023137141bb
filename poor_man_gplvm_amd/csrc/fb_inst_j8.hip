// Scan kernel instances for 8 latent(s) per lane (see fb_kernels.h).
#include "fb_kernels.h"

namespace pmg {
PMG_FB_INSTANCES(8)
}  // namespace pmg
