"""Parity-check matrices and device graphs.

HMatrix mirrors the reference's H_matrix (src/array_and_matrix_operations.hpp:
60-77) as flat CSR (check_nodes) + CSC (bit_nodes) arrays; load_matrix() calls
the C ABI's reader, which restates the reference's four file formats.
Graph owns a qldpc_graph: the decoder's lane partition, replicated on devices.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import Params, check, lib, ptr


@dataclass
class HMatrix:
    n: int
    m: int
    row_ptr: np.ndarray  # int32[m+1] check_nodes
    col_idx: np.ndarray  # int32[nnz]
    col_ptr: np.ndarray  # int32[n+1] bit_nodes
    row_idx: np.ndarray  # int32[nnz]
    is_regular: bool = False

    @property
    def nnz(self) -> int:
        return int(self.row_ptr[-1])

    @property
    def check_nodes(self) -> list[list[int]]:
        rp, ci = self.row_ptr, self.col_idx
        return [ci[rp[j]:rp[j + 1]].tolist() for j in range(self.m)]

    @property
    def bit_nodes(self) -> list[list[int]]:
        cp, ri = self.col_ptr, self.row_idx
        return [ri[cp[i]:cp[i + 1]].tolist() for i in range(self.n)]

    @property
    def code_rate(self) -> float:
        """1 - M/N (reference src/simulation.cpp:389)."""
        return 1.0 - self.m / self.n

    @classmethod
    def from_check_nodes(cls, n: int, check_nodes: list[list[int]]) -> "HMatrix":
        """H from per-check bit lists; bit_nodes is the ascending transpose."""
        m = len(check_nodes)
        row_ptr = np.zeros(m + 1, np.int32)
        row_ptr[1:] = np.cumsum([len(r) for r in check_nodes])
        col_idx = np.array([c for r in check_nodes for c in r], np.int32)
        order = np.lexsort((np.repeat(np.arange(m), np.diff(row_ptr)), col_idx))
        row_idx = np.repeat(np.arange(m, dtype=np.int32), np.diff(row_ptr))[order]
        col_ptr = np.zeros(n + 1, np.int32)
        col_ptr[1:] = np.cumsum(np.bincount(col_idx, minlength=n))
        return cls(n, m, row_ptr, col_idx, col_ptr, row_idx.astype(np.int32), False)

    def syndrome(self, bits: np.ndarray) -> np.ndarray:
        """calculate_syndrome over the last axis (src/array_and_matrix_operations.cpp:936-950)."""
        b = np.asarray(bits, np.uint8)
        vals = b[..., self.col_idx].astype(np.int64)
        cs = np.concatenate([np.zeros(b.shape[:-1] + (1,), np.int64), np.cumsum(vals, axis=-1)], axis=-1)
        # (advanced indexing on the last axis yields a Fortran-ordered result: make it row-major)
        return np.ascontiguousarray(((cs[..., self.row_ptr[1:]] - cs[..., self.row_ptr[:-1]]) & 1).astype(np.uint8))


def load_matrix(path: str, fmt: int) -> HMatrix:
    """Read a matrix file in reference format `fmt` (0 uncompressed, 1 alist, 2 sparse_1, 3 sparse_2)."""
    L = lib()
    n, m, nnz, reg = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    p = str(path).encode()
    check(L.qldpc_load_matrix(p, fmt, ctypes.byref(n), ctypes.byref(m), ctypes.byref(nnz), None, None, None, None,
                              ctypes.byref(reg)), f"qldpc_load_matrix({path})")
    rp = np.empty(m.value + 1, np.int32)
    ci = np.empty(nnz.value, np.int32)
    cp = np.empty(n.value + 1, np.int32)
    ri = np.empty(nnz.value, np.int32)
    check(L.qldpc_load_matrix(p, fmt, ctypes.byref(n), ctypes.byref(m), ctypes.byref(nnz), ptr(rp), ptr(ci), ptr(cp),
                              ptr(ri), ctypes.byref(reg)), f"qldpc_load_matrix({path})")
    return HMatrix(n.value, m.value, rp, ci, cp, ri, bool(reg.value))


@dataclass
class DecodeOutput:
    bits: np.ndarray        # uint8[batch, n]  bit_array_out
    iterations: np.ndarray  # uint32[batch]    decoding_result.iterations_num
    synd_ok: np.ndarray     # uint8[batch]     decoding_result.syndromes_match
    posterior: np.ndarray | None  # float64[batch, n] total_bit_llr


@dataclass
class TrialsOutput:
    iterations: np.ndarray  # uint32[count] decoding_result.iterations_num
    synd_ok: np.ndarray     # uint8[count]  decoding_result.syndromes_match
    keys_match: np.ndarray  # uint8[count]  LDPC_result.keys_match
    runtime_us: np.ndarray  # float64[count] trial_result.runtime (share of the chunk window, see the C ABI)
    accurate_qber: float    # trial_result.accurate_QBER (the same for every trial)


class TrialsJob:
    """One combination's trials in flight (qldpc_run_trials_submit); keeps the
    graph, the rate plan and the output arrays alive until wait()."""

    def __init__(self, graph, plan, count: int):
        self.graph, self.plan, self.handle = graph, plan, None
        self.it = np.empty(count, np.uint32)
        self.ok = np.empty(count, np.uint8)
        self.km = np.empty(count, np.uint8)
        self.rt = np.empty(count, np.float64)
        self.q = ctypes.c_double(0.0)
        self._out = None

    def wait(self) -> TrialsOutput:
        if self._out is None:
            h, self.handle = self.handle, None
            check(lib().qldpc_run_trials_wait(h), "qldpc_run_trials_wait")
            self._out = TrialsOutput(self.it, self.ok, self.km, self.rt, self.q.value)
        return self._out

    def __del__(self):
        if self.handle is not None:  # a job is always completed (its slots hold our arrays)
            try:
                lib().qldpc_run_trials_wait(self.handle)
            except Exception:
                pass


def _canonical_adjacency(H: HMatrix) -> bool:
    """check_nodes rows ascending and bit_nodes their ascending transpose: the
    reference's slot pairing is then the edge itself (src/qkd_ldpc_algorithm.cpp:
    67-69,116-118)."""
    rp, ci = np.asarray(H.row_ptr), np.asarray(H.col_idx)
    rows = np.repeat(np.arange(H.m, dtype=np.int64), np.diff(rp))
    if ci.size and np.any((np.diff(ci) <= 0) & (rows[1:] == rows[:-1])):
        return False
    order = np.lexsort((rows, ci))
    cp = np.zeros(H.n + 1, np.int64)
    np.add.at(cp, ci.astype(np.int64) + 1, 1)
    return np.array_equal(np.cumsum(cp), np.asarray(H.col_ptr)) and np.array_equal(rows[order], np.asarray(H.row_idx))


class Graph:
    """A device-resident Tanner graph (qldpc_graph).

    device_mask: replicate on these HIP devices (bit d = device d; 0 = the
    current one).  devices: an explicit list instead, one shard per entry
    (a device may repeat: concurrent shards on one GPU); decode() then splits a
    batch in len(devices) contiguous slices, one host thread each.
    host_only: plan without touching a device (inspection; cannot decode)."""

    def __init__(self, H: HMatrix, device_mask: int = 0, devices=None, host_only: bool = False):
        self.H = H
        self.n, self.m = H.n, H.m
        g = ctypes.c_void_p()
        self.host_only = bool(host_only)
        if host_only and not _canonical_adjacency(H):
            # (the host-only planner takes check_nodes only and assumes bit_nodes
            # is their ascending transpose; the reference's occurrence pairing of
            # other lists needs qldpc_graph_create_checked)
            raise ValueError("unsorted adjacency: use Graph(H) / Graph(H, devices=...)")
        if host_only:
            check(lib().qldpc_graph_create_host(H.n, H.m, ptr(H.row_ptr), ptr(H.col_idx), ctypes.byref(g)),
                  "qldpc_graph_create_host")
        elif devices is not None:
            dl = np.ascontiguousarray(devices, np.int32)
            check(lib().qldpc_graph_create_checked_on(H.n, H.m, ptr(H.row_ptr), ptr(H.col_idx), ptr(H.col_ptr),
                                                      ptr(H.row_idx), ptr(dl), int(dl.size), ctypes.byref(g)),
                  "qldpc_graph_create_checked_on")
        else:
            check(lib().qldpc_graph_create_checked(H.n, H.m, ptr(H.row_ptr), ptr(H.col_idx), ptr(H.col_ptr),
                                                   ptr(H.row_idx), int(device_mask), ctypes.byref(g)),
                  "qldpc_graph_create_checked")
        self._g = g

    def labels(self) -> tuple[np.ndarray, dict]:
        """The decoder's bank-aware label of each bit id, and the relabelling stats."""
        lab = np.empty(self.n, np.int32)
        st = np.zeros(4, np.int64)
        check(lib().qldpc_graph_labels(self._g, ptr(lab), ptr(st)), "qldpc_graph_labels")
        return lab, {"excess_before": int(st[0]), "excess_after": int(st[1]), "cycles_before": int(st[2]),
                     "cycles_after": int(st[3])}

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._g

    def close(self) -> None:
        if getattr(self, "_g", None) is not None and self._g.value:
            lib().qldpc_graph_destroy(self._g)
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self) -> dict:
        n, m, nnz, nd = (ctypes.c_int32() for _ in range(4))
        check(lib().qldpc_graph_info(self._g, ctypes.byref(n), ctypes.byref(m), ctypes.byref(nnz), ctypes.byref(nd)),
              "qldpc_graph_info")
        return {"n": n.value, "m": m.value, "nnz": nnz.value, "devices": nd.value}

    def plan(self, device: int = 0, algorithm: int = 0) -> dict:
        """Launch geometry; a host-only graph has no device, so workgroups is None."""
        lanes, epl, wgs, lds = (ctypes.c_int32() for _ in range(4))
        var = ctypes.c_char_p()
        check(lib().qldpc_graph_plan(self._g, device, algorithm, ctypes.byref(lanes), ctypes.byref(epl),
                                     None if self.host_only else ctypes.byref(wgs), ctypes.byref(lds),
                                     ctypes.byref(var)), "qldpc_graph_plan")
        return {"lanes": lanes.value, "edges_per_lane": epl.value,
                "workgroups": None if self.host_only else wgs.value,
                "lds_bytes": lds.value, "variant": var.value.decode()}

    def split_plan(self) -> dict:
        """Split-frame shape (qldpc_graph_split_plan): parts per frame, lanes per
        part, scratch message slots per lane (parts == 1: one workgroup per frame)."""
        k, pl, rg = (ctypes.c_int32() for _ in range(3))
        check(lib().qldpc_graph_split_plan(self._g, ctypes.byref(k), ctypes.byref(pl), ctypes.byref(rg)),
              "qldpc_graph_split_plan")
        return {"parts": k.value, "part_lanes": pl.value, "scratch_slots": rg.value}

    def set_kernel_timing(self, enabled: bool = True) -> None:
        """Bracket every decode kernel launch with HIP events (qldpc_set_kernel_timing)."""
        check(lib().qldpc_set_kernel_timing(self._g, 1 if enabled else 0), "qldpc_set_kernel_timing")

    def last_decode_kernel_ms(self, stream=None, device: int = 0) -> float:
        """Duration of the last timed decode kernel on (device, stream); waits for it."""
        ms = ctypes.c_float(0.0)
        check(lib().qldpc_last_decode_kernel_ms(self._g, device, _stream_ptr(stream, device), ctypes.byref(ms)),
              "qldpc_last_decode_kernel_ms")
        return float(ms.value)

    def last_claim_order(self, stream=None, device: int = 0, cap: int = 1 << 20):
        """(order, weight) of the last decode on (device, stream): the claim
        order and each frame's weight, or (None, None) for index order."""
        order = np.empty(cap, np.int32)
        weight = np.empty(cap, np.int32)
        cnt = ctypes.c_int32(0)
        check(lib().qldpc_last_claim_order(self._g, device, _stream_ptr(stream, device), order.ctypes.data,
                                           weight.ctypes.data, cap, ctypes.byref(cnt)), "qldpc_last_claim_order")
        if cnt.value == 0:
            return None, None
        return order[:cnt.value].copy(), weight[:cnt.value].copy()

    # ---- host-buffer decode (synchronous, shards over the graph's devices) ----
    def decode(self, params: Params, llr: np.ndarray, syndrome: np.ndarray, posterior: bool = False) -> DecodeOutput:
        llr = np.ascontiguousarray(llr, np.float64)
        syn = np.ascontiguousarray(syndrome, np.uint8)
        if llr.ndim == 1:
            llr = llr[None, :]
        if syn.ndim == 1:
            syn = syn[None, :]
        batch = llr.shape[0]
        if llr.shape != (batch, self.n) or syn.shape != (batch, self.m):
            raise ValueError(f"expected llr ({batch},{self.n}) and syndrome ({batch},{self.m})")
        bits = np.empty((batch, self.n), np.uint8)
        iters = np.empty(batch, np.uint32)
        ok = np.empty(batch, np.uint8)
        post = np.empty((batch, self.n), np.float64) if posterior else None
        p = params.c()
        check(lib().qldpc_decode_batch(self._g, ctypes.byref(p), batch, ptr(llr), ptr(syn), ptr(bits), ptr(iters),
                                       ptr(ok), ptr(post)), "qldpc_decode_batch")
        return DecodeOutput(bits, iters, ok, post)

    # ---- device-pointer entries (torch tensors as plumbing) ----
    def decode_device(self, params: Params, llr, syndrome, bits, iters, ok, posterior=None, stream=None,
                      device: int | None = None) -> None:
        dev = llr.device.index if device is None else device
        p = params.c()
        check(lib().qldpc_decode_batch_device(
            self._g, dev, ctypes.byref(p), int(llr.shape[0]), _dp(llr), _dp(syndrome), _dp(bits),
            _dp(iters), _dp(ok), _dp(posterior),
            _stream_ptr(stream, dev)), "qldpc_decode_batch_device")

    def build_frames_device(self, alice, bob, log_p, llr, syndrome, stream=None, device: int | None = None) -> None:
        dev = alice.device.index if device is None else device
        check(lib().qldpc_build_frames_device(self._g, dev, int(alice.shape[0]), _dp(alice), _dp(bob),
                                              _dp(log_p), _dp(llr), _dp(syndrome),
                                              _stream_ptr(stream, dev)), "qldpc_build_frames_device")

    def qkd_ldpc_device(self, params: Params, alice, bob, log_p, llr_ws, synd_ws, bits, iters, ok, keys_match,
                        stream=None, device: int | None = None) -> None:
        """QKD_LDPC's per-trial window for a batch, all on device."""
        dev = alice.device.index if device is None else device
        p = params.c()
        check(lib().qldpc_qkd_ldpc_batch_device(
            self._g, dev, ctypes.byref(p), int(alice.shape[0]), _dp(alice), _dp(bob), _dp(log_p),
            _dp(llr_ws), _dp(synd_ws), _dp(bits), _dp(iters), _dp(ok),
            _dp(keys_match), _stream_ptr(stream, dev)), "qldpc_qkd_ldpc_batch_device")


    # ---- the simulation loop's batch seam (host pointers; shards over the devices) ----
    def run_trials(self, params: Params, qber: float, seeds, seed_add: int = 0, plan: "RatePlan | None" = None):
        """run_trial for every seed (src/simulation.cpp:540-576; seed = seeds[t] +
        seed_add) on device through qldpc_run_trials.  -> TrialsOutput."""
        sd = np.ascontiguousarray(seeds, np.uint64)
        cnt = int(sd.size)
        it = np.empty(cnt, np.uint32)
        ok = np.empty(cnt, np.uint8)
        km = np.empty(cnt, np.uint8)
        rt = np.empty(cnt, np.float64)
        q = ctypes.c_double(0.0)
        p = params.c()
        check(lib().qldpc_run_trials(self._g, None if plan is None else plan.handle, ctypes.byref(p), float(qber),
                                     cnt, sd.ctypes.data, int(seed_add) & 0xFFFFFFFFFFFFFFFF, it.ctypes.data,
                                     ok.ctypes.data, km.ctypes.data, rt.ctypes.data, ctypes.byref(q)),
              "qldpc_run_trials")
        return TrialsOutput(it, ok, km, rt, q.value)

    def submit_trials(self, params: Params, qber: float, seeds, seed_add: int = 0,
                      plan: "RatePlan | None" = None) -> "TrialsJob":
        """run_trials in two halves (qldpc_run_trials_submit / _wait): the trials
        are on the devices when this returns; TrialsJob.wait() -> TrialsOutput.
        Lets a driver put the next combination on the GPUs before it collects
        this one."""
        sd = np.ascontiguousarray(seeds, np.uint64)
        cnt = int(sd.size)
        job = TrialsJob(self, plan, cnt)
        p = params.c()
        h = ctypes.c_void_p()
        check(lib().qldpc_run_trials_submit(self._g, None if plan is None else plan.handle, ctypes.byref(p),
                                            float(qber), cnt, sd.ctypes.data, int(seed_add) & 0xFFFFFFFFFFFFFFFF,
                                            job.it.ctypes.data, job.ok.ctypes.data, job.km.ctypes.data,
                                            job.rt.ctypes.data, ctypes.byref(job.q), ctypes.byref(h)),
              "qldpc_run_trials_submit")
        job.handle = h
        return job

    def rate_plan(self, punctured, shortened) -> "RatePlan":
        return RatePlan(self, punctured, shortened)

    def qkd_ldpc_rate_adapt_device(self, plan: "RatePlan", params: Params, alice, bob, punct_alice, punct_bob, log_p,
                                   alice_ext, llr_ws, synd_ws, bits, iters, ok, keys_match, stream=None,
                                   device: int | None = None) -> None:
        """QKD_LDPC_RATE_ADAPT's per-trial window for a batch, all on device."""
        dev = alice.device.index if device is None else device
        p = params.c()
        check(lib().qldpc_qkd_ldpc_rate_adapt_batch_device(
            self._g, plan.handle, dev, ctypes.byref(p), int(alice.shape[0]), _dp(alice), _dp(bob),
            _dp(punct_alice), _dp(punct_bob), _dp(log_p), _dp(alice_ext), _dp(llr_ws),
            _dp(synd_ws), _dp(bits), _dp(iters), _dp(ok), _dp(keys_match),
            _stream_ptr(stream, dev)), "qldpc_qkd_ldpc_rate_adapt_batch_device")

    def build_frames_rate_adapt_device(self, plan: "RatePlan", alice, bob, punct_alice, punct_bob, log_p, alice_ext,
                                       llr, syndrome, stream=None, device: int | None = None) -> None:
        dev = alice.device.index if device is None else device
        check(lib().qldpc_build_frames_rate_adapt_device(
            self._g, plan.handle, dev, int(alice.shape[0]), _dp(alice), _dp(bob), _dp(punct_alice),
            _dp(punct_bob), _dp(log_p), _dp(alice_ext), _dp(llr), _dp(syndrome),
            _stream_ptr(stream, dev)), "qldpc_build_frames_rate_adapt_device")


class RatePlan:
    """Punctured / shortened positions of one adapted rate, on the graph's devices."""

    def __init__(self, graph: Graph, punctured, shortened):
        self.punctured = np.ascontiguousarray(punctured, np.int32)
        self.shortened = np.ascontiguousarray(shortened, np.int32)
        h = ctypes.c_void_p()
        check(lib().qldpc_rate_plan_create(graph.handle, self.punctured.size, self.punctured.ctypes.data,
                                           self.shortened.size, self.shortened.ctypes.data, ctypes.byref(h)),
              "qldpc_rate_plan_create")
        self.handle = h
        self._graph = graph  # keep the graph alive

    def __del__(self):
        if getattr(self, "handle", None) is not None and self.handle.value:
            lib().qldpc_rate_plan_destroy(self.handle)
            self.handle = None


def keys_match_device(alice, bits, out, stream=None) -> None:
    dev = alice.device.index
    check(lib().qldpc_keys_match_device(int(alice.shape[0]), int(alice.shape[1]), _dp(alice), _dp(bits),
                                        _dp(out), _stream_ptr(stream, dev)), "qldpc_keys_match_device")


def trial_seeds(simulation_seed: int, count: int) -> np.ndarray:
    """Per-trial seeds of the simulation loop (src/simulation.cpp:713-719)."""
    out = np.empty(count, np.uint64)
    check(lib().qldpc_trial_seeds(int(simulation_seed) & 0xFFFFFFFFFFFFFFFF, int(count), out.ctypes.data),
          "qldpc_trial_seeds")
    return out


def trials_device(n: int, qber: float, seeds, alice, bob, seed_add: int = 0, stream=None) -> float:
    """run_trial's keys for every seed, on device (src/simulation.cpp:540-551).
    seeds: device uint64 tensor [batch]; alice/bob: device uint8 [batch, n].
    Returns the accurate QBER floor(n*qber)/n."""
    import ctypes

    dev = seeds.device.index
    q = ctypes.c_double(0.0)
    check(lib().qldpc_trials_device(int(n), float(qber), int(seeds.shape[0]), _dp(seeds),
                                    int(seed_add) & 0xFFFFFFFFFFFFFFFF, _dp(alice), _dp(bob),
                                    ctypes.byref(q), _stream_ptr(stream, dev)), "qldpc_trials_device")
    return q.value


def xoshiro_state(seed: int) -> np.ndarray:
    st = np.empty(4, np.uint64)
    check(lib().qldpc_xoshiro_state(int(seed) & 0xFFFFFFFFFFFFFFFF, st.ctypes.data), "qldpc_xoshiro_state")
    return st


def adapt_code_rate(n: int, m: int, qber: float, delta: float, efficiency: float, untainted=None, state=None):
    """adapt_code_rate (src/array_and_matrix_operations.cpp:1131-1223).
    state: np.uint64[4] generator state, advanced in place (chain calls like the
    reference's setup loop).  -> (punctured, shortened, adapted_rate); empty
    lists for the reference's skipped (out-of-range) combinations."""
    import ctypes

    if state is None:
        raise ValueError("pass the generator state (xoshiro_state(seed))")
    unt = None if untainted is None else np.ascontiguousarray(untainted, np.int32)
    p = np.empty(n, np.int32)
    s = np.empty(n, np.int32)
    npn, nsn = ctypes.c_int32(0), ctypes.c_int32(0)
    rate = ctypes.c_double(0.0)
    check(lib().qldpc_adapt_code_rate(n, m, qber, delta, efficiency, 0 if unt is None else 1,
                                      None if unt is None else unt.ctypes.data, 0 if unt is None else unt.size,
                                      state.ctypes.data, p.ctypes.data, ctypes.byref(npn), s.ctypes.data,
                                      ctypes.byref(nsn), ctypes.byref(rate)), "qldpc_adapt_code_rate")
    return p[:npn.value].copy(), s[:nsn.value].copy(), rate.value


def select_punctured_untainted(H: "HMatrix", state) -> np.ndarray:
    """select_punctured_bits_untainted (src/array_and_matrix_operations.cpp:
    1002-1067): the untainted puncturing list in selection order — what the
    reference writes to a missing .untp file (:1076-1123).  state: np.uint64[4]
    generator state (xoshiro_state(seed)), advanced in place."""
    import ctypes

    if state is None:
        raise ValueError("pass the generator state (xoshiro_state(seed))")
    rp, ci = np.ascontiguousarray(H.row_ptr, np.int32), np.ascontiguousarray(H.col_idx, np.int32)
    cp, ri = np.ascontiguousarray(H.col_ptr, np.int32), np.ascontiguousarray(H.row_idx, np.int32)
    out = np.empty(H.n, np.int32)
    cnt = ctypes.c_int32(0)
    check(lib().qldpc_select_punctured_untainted(H.n, H.m, rp.ctypes.data, ci.ctypes.data, cp.ctypes.data,
                                                  ri.ctypes.data, state.ctypes.data, out.ctypes.data,
                                                  ctypes.byref(cnt)), "qldpc_select_punctured_untainted")
    return out[:cnt.value].copy()


def trials_rate_adapt_device(n: int, qber: float, seeds, n_punct: int, alice, bob, punct_alice, punct_bob,
                             seed_add: int = 0, stream=None) -> float:
    """trials_device plus QKD_LDPC_RATE_ADAPT's punctured draws (2 per position)."""
    import ctypes

    dev = seeds.device.index
    q = ctypes.c_double(0.0)
    check(lib().qldpc_trials_rate_adapt_device(int(n), float(qber), int(seeds.shape[0]), _dp(seeds),
                                               int(seed_add) & 0xFFFFFFFFFFFFFFFF, int(n_punct), _dp(alice),
                                               _dp(bob), _dp(punct_alice), _dp(punct_bob),
                                               ctypes.byref(q), _stream_ptr(stream, dev)),
          "qldpc_trials_rate_adapt_device")
    return q.value


def _dp(t):
    """Device pointer of a row-major (C-contiguous) tensor: the C ABI reads
    frames as [frame][bit] rows, so a transposed view would be misread."""
    if t is None:
        return None
    if not t.is_contiguous():
        raise ValueError(f"device buffers must be C-contiguous (row-major); got shape {tuple(t.shape)} "
                         f"strides {t.stride()}")
    return t.data_ptr()


def _stream_ptr(stream, device: int):
    if stream is None:
        import torch

        return torch.cuda.current_stream(device).cuda_stream
    return getattr(stream, "cuda_stream", stream)
