// bm_strip_lr.hip — the strip kernel's instantiations with the right view (bm_strip.hip, RIGHT = true), in their
// own translation unit so that the two halves compile in parallel.
#define SM_STRIP_RIGHT_TU 1
#include "bm_strip.hip"
