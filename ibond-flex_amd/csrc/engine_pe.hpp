// Host interface of the public-key split-pair encryption unit (engine_pe.hip, kernels_pe.hpp).
#pragma once
#include "engine_dec4.hpp"
#include "kernels_pe.hpp"

namespace fpai {

int pe_geometry(int cus, long long chunk, Dec4Geom* g);   // gx_pre, gx_pow, gx_L (= k_pe_fin), scratch_bytes
hipError_t pe_launch(const PeParams& p, const Dec4Geom& g, hipStream_t st, hipEvent_t* ev);
// the factored chain's stages (kernels_pe.hpp): k_pe_pre + k_pe_awords (then the caller's batch inversion of p.aw),
// then k_pe_iota + k_pe_pow_f + k_pe_fin; ev[0..3] nullable (ev[1] before k_pe_pow_f)
hipError_t pe_launch_pre_aw(const PeParams& p, const Dec4Geom& g, hipStream_t st, hipEvent_t* ev);
hipError_t pe_launch_iota_pow_f(const PeParams& p, const Dec4Geom& g, hipStream_t st, hipEvent_t* ev);
// the general chain after pe_launch_pre_aw (a chunk whose batch inversion found a non-unit): k_pe_pow + k_pe_fin
// k_pe_fin alone: c = A + n B from the pairs in p.xw (the public fixed-base path, engine_pfb.hip)
hipError_t pe_launch_fin(const PeParams& p, int cus, hipStream_t st);

}  // namespace fpai
