// gsr_render_fwd.hip -- the forward half of gsr_render.hip (forward blend, tile schedule,
// activations) as its own translation unit, so that it can be compiled with other flags than the
// backward (Makefile FLAGS_gsr_render_fwd.hip).
#define GSR_RENDER_PART 2
#include "gsr_render.hip"
