// piadmm_device_spec.hip -- the speculative loop shape's instantiations of k_mpc_step (piadmm_device.hip
// with PIADMM_SPEC_TU): a kernel of their own, so that the register allocation of the speculative
// shape's hot loops is not shaped by the plain shape's code (and the two compile in parallel).
#define PIADMM_SPEC_TU 1
#include "piadmm_device.hip"
