// mgqp_ctl.h — the opaque handle behind include/mgqp_amd.h (shared by the C-ABI files).
#ifndef MGQP_CTL_H
#define MGQP_CTL_H
#include "quadprog_amd/mgqp.hh"

struct mgqp_ctl {
  mgqp_amd::MotionGenerationQuadraticProgram c;
};

extern "C" void mgqp_capi_set_error(const char* msg);

#endif
