// The fused 8-schools kernel's zero-padding form (4 chains per wave, Dp = 16) in a translation
// unit of its own, built with LLVM's iterative ILP scheduling strategy (Makefile; nuts.hip's
// launch_fused_ut calls it through stk_launch_fused4_zp).
#define STK_NUTS_FUSED4_TU
#include "nuts.hip"
