"""qkd_ldpc_v_amd — MI355X (gfx950) LDPC belief-propagation decoding for QKD.

The product is libqkdldpc_hip.so (HIP kernels + C ABI, include/qkd_ldpc_hip.h);
this package binds it and mirrors the reference's decode interface
(ColdCloudd/QKD_LDPC_V src/qkd_ldpc_algorithm.hpp).
"""
from ._lib import (ALGORITHM_NAMES, ANMSA, AOMSA, NMSA, OMSA, SPA, SPA_LIN, Params, QLDPCError, exported_symbols, lib,
                   log_p, version)
from .graph import (DecodeOutput, Graph, HMatrix, RatePlan, TrialsOutput, adapt_code_rate, keys_match_device, load_matrix,
                    select_punctured_untainted,
                    trial_seeds, trials_device, trials_rate_adapt_device, xoshiro_state)
from .trials import bsc_frames
from .codes import regular_code

__all__ = [
    "regular_code",
    "ALGORITHM_NAMES", "ANMSA", "AOMSA", "NMSA", "OMSA", "SPA", "SPA_LIN", "Params", "QLDPCError",
    "exported_symbols", "lib", "log_p", "version", "DecodeOutput", "TrialsOutput", "Graph", "HMatrix", "keys_match_device",
    "trial_seeds", "trials_device", "RatePlan", "adapt_code_rate", "trials_rate_adapt_device", "xoshiro_state",
    "load_matrix", "bsc_frames",
]
