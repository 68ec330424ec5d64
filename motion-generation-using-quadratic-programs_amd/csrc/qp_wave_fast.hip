// qp_wave_fast.hip — the QPGPU_FLAG_FAST build of the LDS variants of qp_wave.hip (n <= 64,
// m <= 256): the same source with QPGPU_WAVE_FAST=1, built with -ffp-contract=fast (Makefile).
// See qp_wave.hip's header and DESIGN §5.7.
#define QPGPU_WAVE_FAST 1
#include "qp_wave.hip"
