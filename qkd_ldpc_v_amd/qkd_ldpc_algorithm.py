"""Reference-named decode interface (Python mirror of src/qkd_ldpc_algorithm.hpp).

Same names, argument meaning and results as ColdCloudd/QKD_LDPC_V:
  decoding_result / LDPC_result          src/qkd_ldpc_algorithm.hpp:16-26
  the six decoders                       src/qkd_ldpc_algorithm.hpp:28-90
  QKD_LDPC                               src/qkd_ldpc_algorithm.cpp:1031-1119
  calculate_syndrome / arrays_equal / remove_bits
                                         src/array_and_matrix_operations.cpp:105-118,259-287,936-950
  read_sparse_*                          src/array_and_matrix_operations.cpp:291-886
The hidden global-CFG inputs (algorithm choice, iteration cap, LLR threshold
switch) live in CFG, as in the reference.  Every decode runs on the GPU through
libqkdldpc_hip.so; the batched form is decode_batch().
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from ._lib import ANMSA, AOMSA, NMSA, OMSA, SPA, SPA_LIN, Params, log_p
from .graph import Graph, HMatrix, load_matrix

DEC_SPA, DEC_SPA_APPROX, DEC_NMSA, DEC_OMSA, DEC_ANMSA, DEC_AOMSA = SPA, SPA_LIN, NMSA, OMSA, ANMSA, AOMSA
ALMOST_ZERO = 1e-4  # src/qkd_ldpc_algorithm.hpp:13


@dataclass
class ConfigData:
    """The config_data fields the decode path reads (src/config.hpp:103-196)."""

    DECODING_ALGORITHM: int = DEC_SPA
    DECODING_ALG_MAX_ITERATIONS: int = 50
    ENABLE_DECODING_ALG_MSG_LLR_THRESHOLD: bool = True
    DECODING_ALG_MSG_LLR_THRESHOLD: float = 100.0
    ENABLE_PRIVACY_MAINTENANCE: bool = False


CFG = ConfigData()


@dataclass
class decoding_result:  # noqa: N801 — reference name
    iterations_num: int = 0
    syndromes_match: bool = False


@dataclass
class LDPC_result:  # noqa: N801
    decoding_res: decoding_result = field(default_factory=decoding_result)
    keys_match: bool = False


@dataclass
class decoding_scaling_factors:  # noqa: N801
    primary: float = 0.0
    secondary: float = 0.0


@dataclass
class H_matrix_params:  # noqa: N801
    bits_to_remove: list = field(default_factory=list)
    punctured_bits: list = field(default_factory=list)
    shortened_bits: list = field(default_factory=list)


def read_sparse_uncompressed_matrix(path) -> HMatrix:
    return load_matrix(path, 0)


def read_sparse_matrix_alist(path) -> HMatrix:
    return load_matrix(path, 1)


def read_sparse_matrix_1(path) -> HMatrix:
    return load_matrix(path, 2)


def read_sparse_matrix_2(path) -> HMatrix:
    return load_matrix(path, 3)


def calculate_syndrome(bit_array, matrix: HMatrix, syndrome_out=None) -> np.ndarray:
    s = matrix.syndrome(np.asarray(bit_array, np.uint8))
    if syndrome_out is not None:
        syndrome_out[:] = s
    return s


def arrays_equal(array1, array2) -> bool:
    a = np.asarray(array1)
    return bool(np.array_equal(a, np.asarray(array2)[: a.shape[0]]))


def remove_bits(bits_to_remove, array1, array2):
    keep = np.ones(len(array1), bool)
    keep[np.asarray(bits_to_remove, np.int64)] = False
    return np.asarray(array1)[keep], np.asarray(array2)[keep]


_graphs: dict[int, Graph] = {}


def _graph(matrix: HMatrix) -> Graph:
    g = _graphs.get(id(matrix))
    if g is None or g.H is not matrix:
        g = Graph(matrix)
        _graphs[id(matrix)] = g
    return g


def _decode(alg, bit_array_llr, matrix, syndrome, max_num_iterations, msg_threshold, bit_array_out, primary=0.0,
            secondary=0.0) -> decoding_result:
    p = Params(alg, int(max_num_iterations), bool(CFG.ENABLE_DECODING_ALG_MSG_LLR_THRESHOLD), float(msg_threshold),
               float(primary), float(secondary))
    out = _graph(matrix).decode(p, np.asarray(bit_array_llr, np.float64), np.asarray(syndrome, np.uint8) & 1)
    if bit_array_out is not None:
        bit_array_out[:] = out.bits[0]
    return decoding_result(int(out.iterations[0]), bool(out.synd_ok[0]))


def sum_product_decoding(bit_array_llr, matrix, syndrome, max_num_iterations, msg_threshold, bit_array_out):
    return _decode(SPA, bit_array_llr, matrix, syndrome, max_num_iterations, msg_threshold, bit_array_out)


def sum_product_linear_approx_decoding(bit_array_llr, matrix, syndrome, max_num_iterations, msg_threshold,
                                       bit_array_out):
    return _decode(SPA_LIN, bit_array_llr, matrix, syndrome, max_num_iterations, msg_threshold, bit_array_out)


def min_sum_normalized_decoding(bit_array_llr, matrix, syndrome, max_num_iterations, alpha, msg_threshold,
                                bit_array_out):
    return _decode(NMSA, bit_array_llr, matrix, syndrome, max_num_iterations, msg_threshold, bit_array_out, alpha)


def min_sum_offset_decoding(bit_array_llr, matrix, syndrome, max_num_iterations, beta, msg_threshold, bit_array_out):
    return _decode(OMSA, bit_array_llr, matrix, syndrome, max_num_iterations, msg_threshold, bit_array_out, beta)


def adaptive_min_sum_normalized_decoding(bit_array_llr, matrix, syndrome, max_num_iterations, alpha, nu,
                                         msg_threshold, bit_array_out):
    return _decode(ANMSA, bit_array_llr, matrix, syndrome, max_num_iterations, msg_threshold, bit_array_out, alpha,
                   nu)


def adaptive_min_sum_offset_decoding(bit_array_llr, matrix, syndrome, max_num_iterations, beta, sigma,
                                     msg_threshold, bit_array_out):
    return _decode(AOMSA, bit_array_llr, matrix, syndrome, max_num_iterations, msg_threshold, bit_array_out, beta,
                   sigma)


def QKD_LDPC(matrix: HMatrix, alice_bit_array, bob_bit_array, QBER: float,  # noqa: N802,N803
             scaling_factors: decoding_scaling_factors | None = None,
             matrix_params: H_matrix_params | None = None) -> LDPC_result:
    """One trial (src/qkd_ldpc_algorithm.cpp:1031-1119), decoded on the GPU."""
    sf = scaling_factors or decoding_scaling_factors()
    lp = log_p(QBER)
    bob = np.asarray(bob_bit_array, np.uint8)
    apriori_llr = np.where(bob != 0, -lp, lp)
    alice_syndrome = matrix.syndrome(np.asarray(alice_bit_array, np.uint8))
    bob_solution = np.zeros(matrix.n, np.uint8)
    res = _decode(int(CFG.DECODING_ALGORITHM), apriori_llr, matrix, alice_syndrome, CFG.DECODING_ALG_MAX_ITERATIONS,
                  CFG.DECODING_ALG_MSG_LLR_THRESHOLD, bob_solution, sf.primary, sf.secondary)
    keys = arrays_equal(alice_bit_array, bob_solution)
    if CFG.ENABLE_PRIVACY_MAINTENANCE and matrix_params is not None:
        remove_bits(matrix_params.bits_to_remove, alice_bit_array, bob_solution)
    return LDPC_result(res, keys)


def decode_batch(matrix: HMatrix, llr: np.ndarray, syndrome: np.ndarray,
                 scaling_factors: decoding_scaling_factors | None = None, posterior: bool = False):
    """Batched decode of independent frames with the CFG-selected decoder."""
    sf = scaling_factors or decoding_scaling_factors()
    p = Params(int(CFG.DECODING_ALGORITHM), int(CFG.DECODING_ALG_MAX_ITERATIONS),
               bool(CFG.ENABLE_DECODING_ALG_MSG_LLR_THRESHOLD), float(CFG.DECODING_ALG_MSG_LLR_THRESHOLD),
               sf.primary, sf.secondary)
    return _graph(matrix).decode(p, llr, syndrome, posterior)
