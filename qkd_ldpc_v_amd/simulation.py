"""Config-driven simulation driver on the MI355X pipeline.

Reads the reference's JSON configuration (src/config.cpp:100-400), builds the
same simulation combinations (src/simulation.cpp:178-455: QBER ranges or
rate-adaptation maps x scaling-factor ranges or maps, per matrix), runs every
combination's TRIALS_NUMBER trials on the GPU — the reference's own trial
generator (`seeds[n] + sim_number`, src/simulation.cpp:713-745), device frame
construction, decode and key comparison — aggregates them like
process_trials_results (:580-690) and writes the reference's results CSV
(write_file, :4-176: ';' separated, decimal comma).

    python -m qkd_ldpc_v_amd.simulation CONFIG.json --matrices DIR [--results DIR]

Differences from the reference, by design: the matrix directory is given on
the command line (the reference derives it from matrix_format under its source
tree) and its *.mtrx files are taken in name order (the reference uses
directory order, which the filesystem decides); the untainted-puncturing
search for a missing .untp file runs and writes the file, as the reference's;
the throughput columns' per-trial time is each trial's share of its GPU
chunk's measured window, in proportion to its own decode span (the reference
times each trial's QKD_LDPC call alone on one core; qldpc_run_trials).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import sys
import time
from dataclasses import dataclass, field

import numpy as np

from ._lib import ALGORITHM_NAMES, Params, check, lib
from .graph import Graph, adapt_code_rate, load_matrix, select_punctured_untainted, trial_seeds, xoshiro_state

EPSILON = 1e-6  # src/config.hpp:199
DEC_NAMES = {0: "SPA", 1: "SPA-LIN-APPROX", 2: "NMSA", 3: "OMSA", 4: "ANMSA", 5: "AOMSA"}
FACTOR_KEYS = {  # algorithm -> (config section, primary key, secondary key)
    2: ("min_sum_normalized_parameters", "alpha", None),
    3: ("min_sum_offset_parameters", "beta", None),
    4: ("adaptive_min_sum_normalized_parameters", "alpha", "nu"),
    5: ("adaptive_min_sum_offset_parameters", "beta", "sigma"),
}


class ConfigError(ValueError):
    pass


def _sorted_by_rate(items: list, rate=lambda x: x["code_rate"]) -> list:
    """The reference's std::sort by code_rate (not stable): same permutation."""
    if not items:
        return items
    keys = np.array([rate(x) for x in items], np.float64)
    perm = np.empty(len(items), np.int32)
    check(lib().qldpc_sort_permutation(keys.ctypes.data, len(items), perm.ctypes.data), "qldpc_sort_permutation")
    return [items[i] for i in perm]


def _range(r: dict, what: str) -> dict:
    b, e, s = float(r["begin"]), float(r["end"]), float(r["step"])
    if b <= 0 or e <= 0 or s <= 0:
        raise ConfigError(f"{what} range begin, end, step must be > 0!")
    if b > e:
        raise ConfigError(f"{what} range begin cannot be larger than end!")
    if b != e and s - EPSILON > e - b:
        raise ConfigError(f"{what} range step is too large!")
    return {"begin": b, "end": e, "step": s}


def _range_values(begin: float, end: float, step: float) -> list[float]:
    """begin + j*step, j = 0 .. round((end-begin)/step) (src/simulation.cpp:193-205)."""
    if begin == end:
        return [begin]
    steps = int(round((end - begin) / step)) + 1
    return [begin + float(j) * step for j in range(steps)]


@dataclass
class Config:
    """config_data (src/config.hpp) as the reference parses it."""
    threads_number: int
    trials_number: int
    simulation_seed: int
    enable_privacy_maintenance: bool
    enable_throughput_measurement: bool
    consider_rtt: bool
    rtt: float
    decoding_algorithm: int
    primary: dict = field(default_factory=dict)    # {"use_range", "range" | "maps"}
    secondary: dict = field(default_factory=dict)
    max_iterations: int = 50
    matrix_format: int = 1
    threshold_enabled: bool = True
    threshold: float = 100.0
    qber_ranges: list = field(default_factory=list)
    rate_adaptation: bool = False
    untainted_puncturing: bool = False
    use_adaptation_ranges: bool = False
    adaptation_ranges: list = field(default_factory=list)
    adaptation_maps: list = field(default_factory=list)

    @staticmethod
    def load(path: str) -> "Config":
        with open(path) as f:
            c = json.load(f)
        try:
            return Config._parse(c)
        except KeyError as e:
            raise ConfigError(f"missing configuration parameter {e}") from None

    @staticmethod
    def _parse(c: dict) -> "Config":
        c = _legacy_shim(c)
        if int(c["threads_number"]) < 1:
            raise ConfigError("Number of threads must be > 0!")
        if int(c["trials_number"]) < 1:
            raise ConfigError("Number of trials must be > 0!")
        seed = int(c["simulation_seed"]) if c["use_config_simulation_seed"] else int(time.time())
        tm = bool(c["enable_throughput_measurement"])
        rtt_on, rtt = False, 0.0
        if tm:
            tp = c["throughput_measurement_parameters"]
            rtt_on = bool(tp["consider_RTT"])
            if rtt_on:
                rtt = float(tp["RTT"])
                if rtt < 0:
                    raise ConfigError("RTT must be >= 0!")
        alg = int(c["decoding_algorithm"])
        if alg > 5:
            raise ConfigError("Invalid decoding algorithm.")
        cfg = Config(int(c["threads_number"]), int(c["trials_number"]), seed, bool(c["enable_privacy_maintenance"]),
                     tm, rtt_on, rtt, alg)
        if alg in FACTOR_KEYS:
            sec_name, pk, sk = FACTOR_KEYS[alg]
            ap = c[sec_name]
            for key, slot in ((pk, "primary"), (sk, "secondary")):
                if key is None:
                    continue
                d = {"use_range": bool(ap[f"use_{key}_range"])}
                if d["use_range"]:
                    d["range"] = _range(ap[f"{key}_range"], "Scaling factor")
                else:
                    maps = []
                    for mm in ap[f"code_rate_{key}_maps"]:
                        r, v = float(mm["code_rate"]), float(mm[key])
                        if not 0 < r < 1:
                            raise ConfigError("Code rate(R) must be: 0 < R < 1!")
                        if v <= 0:
                            raise ConfigError("Scaling factor must be > 0!")
                        maps.append({"code_rate": r, "value": v})
                    if not maps:
                        raise ConfigError("Array with code rate(R) and scaling factor maps is empty!")
                    d["maps"] = _sorted_by_rate(maps)
                setattr(cfg, slot, d)
            if sk and not cfg.primary["use_range"] and not cfg.secondary["use_range"]:
                pm, sm = cfg.primary["maps"], cfg.secondary["maps"]
                if len(pm) != len(sm):
                    raise ConfigError(f"{DEC_NAMES[alg]}: The sizes of code_rate_{pk}_maps and code_rate_{sk}_maps "
                                      f"vectors must match! ({len(pm)} vs {len(sm)})")
                for a, b in zip(pm, sm):
                    if abs(a["code_rate"] - b["code_rate"]) > EPSILON:
                        raise ConfigError(f"{DEC_NAMES[alg]}: Mismatch of code_rate in {pk} and {sk} maps")
        cfg.max_iterations = int(c["decoding_algorithm_max_iterations"])
        if cfg.max_iterations < 1:
            raise ConfigError("Maximum number of decoding iterations must be > 0!")
        cfg.matrix_format = int(c["matrix_format"])
        if cfg.matrix_format > 3:
            raise ConfigError("Invalid matrix format.")
        cfg.threshold_enabled = bool(c["enable_decoding_algorithm_msg_llr_threshold"])
        if cfg.threshold_enabled:
            cfg.threshold = float(c["decoding_algorithm_msg_llr_threshold"])
            if cfg.threshold <= 0:
                raise ConfigError("Threshold must be > 0!")
        ranges = []
        for r in c["code_rate_QBER_ranges"]:
            q = r["QBER"]
            e = {"code_rate": float(r["code_rate"]), "begin": float(q["begin"]), "end": float(q["end"]),
                 "step": float(q["step"])}
            if not 0 < e["code_rate"] < 1:
                raise ConfigError("Code rate(R) must be: 0 < R < 1!")
            if not (0 < e["begin"] < 1 and 0 < e["end"] < 1) or e["begin"] > e["end"]:
                raise ConfigError("Invalid QBER range.")
            if e["step"] <= 0:
                raise ConfigError("QBER step must be > 0!")
            if e["begin"] != e["end"] and e["step"] - EPSILON > e["end"] - e["begin"]:
                raise ConfigError("QBER step is too large.")
            ranges.append(e)
        if not ranges:
            raise ConfigError("Array with code rate(R) and QBER ranges is empty!")
        cfg.qber_ranges = _sorted_by_rate(ranges)
        cfg.rate_adaptation = bool(c["enable_code_rate_adaptation"])
        if cfg.rate_adaptation:
            ra = c["code_rate_adaptation_parameters"]
            cfg.untainted_puncturing = bool(ra["enable_untainted_puncturing"])
            cfg.use_adaptation_ranges = bool(ra["use_adaptation_parameters_ranges"])
            if cfg.use_adaptation_ranges:
                rr = []
                for r in ra["code_rate_adaptation_parameters_ranges"]:
                    d, f = r["delta"], r["efficiency"]
                    rr.append({"code_rate": float(r["code_rate"]),
                               "delta": (float(d["begin"]), float(d["end"]), float(d["step"])),
                               "efficiency": (float(f["begin"]), float(f["end"]), float(f["step"]))})
                if not rr:
                    raise ConfigError("Array with code rate(R) and adaptation parameters ranges is empty!")
                for e in rr:  # src/config.cpp:327-354, same order and messages
                    if not 0 < e["code_rate"] < 1:
                        raise ConfigError("Code rate(R) must be: 0 < R < 1!")
                    db, de, ds = e["delta"]
                    if not (0 < db < 1 and 0 < de < 1) or db > de:
                        raise ConfigError("Invalid delta begin or end parameters. Delta must be: 0 < delta < 1, "
                                          "and begin cannot be larger than end!")
                    if not ds > 0:
                        raise ConfigError("Delta step must be > 0!")
                    if db != de and ds - EPSILON > de - db:
                        raise ConfigError("Delta step is too large.")
                    fb, fe, fs = e["efficiency"]
                    if fb < 1 or fe < 1 or fb > fe:
                        raise ConfigError("Invalid efficiency begin or end parameters. Efficiency(f_EC) must be: "
                                          "f_EC >= 1, and begin cannot be larger than end!")
                    if not fs > 0:
                        raise ConfigError("Efficiency step must be > 0!")
                    if fb != fe and fs - EPSILON > fe - fb:
                        raise ConfigError("Efficiency step is too large.")
                cfg.adaptation_ranges = _sorted_by_rate(rr)
            else:
                mm = []
                for m in ra["code_rate_QBER_adaptation_parameters_maps"]:
                    e = {"code_rate": float(m["code_rate"]), "QBER": float(m["QBER"]), "delta": float(m["delta"]),
                         "efficiency": float(m["efficiency"])}
                    if not 0 < e["code_rate"] < 1:
                        raise ConfigError("Code rate(R) must be: 0 < R < 1!")
                    if not 0 < e["QBER"] < 1:
                        raise ConfigError("Invalid QBER parameter. QBER must be: 0 < QBER < 1!")
                    if not 0 < e["delta"] < 1:
                        raise ConfigError("Invalid delta parameter. Delta must be: 0 < delta < 1!")
                    if e["efficiency"] < 1:
                        raise ConfigError("Invalid efficiency parameter. Efficiency(f_EC) must be: f_EC >= 1!")
                    mm.append(e)
                if not mm:
                    raise ConfigError("Array with code rate(R), QBER and adaptation parameters maps is empty!")
                cfg.adaptation_maps = _sorted_by_rate(mm)
        return cfg


def _legacy_shim(c: dict) -> dict:
    """configs_all/*.json predate the current schema: `code_rate_QBER_maps`
    entries {code_rate, QBER_begin, QBER_end, QBER_step} are today's
    `code_rate_QBER_ranges` {code_rate, QBER: {begin, end, step}}; the oldest
    select the decoder with `use_min_sum_normalized_algorithm` (NMSA, else
    SPA); rate adaptation did not exist (off); `interactive_mode` is ignored."""
    c = dict(c)
    if "decoding_algorithm" not in c and "use_min_sum_normalized_algorithm" in c:
        c["decoding_algorithm"] = 2 if c["use_min_sum_normalized_algorithm"] else 0
    if "code_rate_QBER_ranges" not in c and "code_rate_QBER_maps" in c:
        c["code_rate_QBER_ranges"] = [
            {"code_rate": m["code_rate"],
             "QBER": {"begin": m["QBER_begin"], "end": m["QBER_end"], "step": m["QBER_step"]}}
            for m in c["code_rate_QBER_maps"]]
    c.setdefault("enable_code_rate_adaptation", False)
    return c


# ---- combinations (src/simulation.cpp:178-455) --------------------------------
def _rate_qber_values(cfg: Config, rate: float) -> list[float]:
    for r in cfg.qber_ranges:
        if rate <= r["code_rate"]:
            return _range_values(r["begin"], r["end"], r["step"])
    raise ConfigError(f"An error occurred while generating a QBER range based on code rate(R). "
                      f"Matrix code rate, R = {rate}.")


def _factor_values(d: dict, rate: float) -> list[float]:
    if d["use_range"]:
        r = d["range"]
        return _range_values(r["begin"], r["end"], r["step"])
    for m in d["maps"]:
        if rate <= m["code_rate"]:
            return [m["value"]]
    raise ConfigError(f"An error occurred while searching scaling factor value based on code rate(R). "
                      f"Matrix code rate, R = {rate}.")


def _adapt_maps(cfg: Config, rate: float) -> list[tuple]:
    out, target = [], None
    for m in cfg.adaptation_maps:
        if target is None:
            if rate <= m["code_rate"]:
                target = m["code_rate"]
                out.append((m["QBER"], m["delta"], m["efficiency"]))
        elif m["code_rate"] == target:
            out.append((m["QBER"], m["delta"], m["efficiency"]))
        else:
            break
    if not out:
        raise ConfigError(f"An error occurred while generating a QBER - delta - efficiency(f_EC) maps based on "
                          f"code rate(R). Matrix code rate, R = {rate}.")
    return out


def _adapt_ranges(cfg: Config, rate: float) -> tuple[list, list]:
    for r in cfg.adaptation_ranges:
        if rate <= r["code_rate"]:
            return _range_values(*r["delta"]), _range_values(*r["efficiency"])
    raise ConfigError(f"An error occurred while generating a delta range based on code rate(R). R = {rate}.")


@dataclass
class Combination:
    matrix_index: int
    config_qber: float
    primary: float = 0.0
    secondary: float = 0.0
    punctured: np.ndarray | None = None
    shortened: np.ndarray | None = None
    delta: float = 0.0
    efficiency: float = 0.0
    adapted_rate: float = 0.0
    bits_to_remove: int = 0


def _bits_to_remove(H, punct=None, short=None) -> int:
    cnt = ctypes.c_int32(0)
    p = np.ascontiguousarray(punct if punct is not None else np.empty(0), np.int32)
    s = np.ascontiguousarray(short if short is not None else np.empty(0), np.int32)
    cp = np.ascontiguousarray(H.col_ptr, np.int32)
    ri = np.ascontiguousarray(H.row_idx, np.int32)
    check(lib().qldpc_bits_to_remove(H.n, H.m, cp.ctypes.data, ri.ctypes.data, p.size, p.ctypes.data, s.size,
                                     s.ctypes.data, 1 if punct is not None else 0, None, ctypes.byref(cnt)),
          "qldpc_bits_to_remove")
    return cnt.value


def _punctured_bits_untainted(path: str, H, state) -> np.ndarray:
    """get_punctured_bits_untainted (src/array_and_matrix_operations.cpp:
    1076-1123): the first line of the .untp file next to the matrix; when it is
    missing or empty, the untainted search (select_punctured_untainted, drawing
    from the setup generator `state`) and the file written as the reference
    writes it (indices separated by spaces, one line)."""
    up = os.path.splitext(path)[0] + ".untp"
    unt = np.empty(0, np.int32)
    if os.path.exists(up):
        with open(up) as f:
            unt = np.array(f.readline().split(), np.int64)
    for v in unt:
        if v < 0 or v >= H.n:
            raise ConfigError(f"The punctured bit index '{v}' is out of range [0,{H.n - 1}]. File: {up}")
    if unt.size == 0:
        print(f"WARNING: No file with punctured untainted bits found: {up} \nThis file will be automatically "
              "created. Wait...", file=sys.stderr)
        unt = select_punctured_untainted(H, state)
        try:
            with open(up, "w") as f:
                f.write("".join(f"{int(v)} " for v in unt))
        except OSError as e:
            raise ConfigError(f"Unable to open file for writing: {up}") from e
        print("File created successfully.", file=sys.stderr)
    return unt.astype(np.int32)


def prepare(cfg: Config, matrix_paths: list[str]):
    """prepare_sim_inputs (src/simulation.cpp:394-455): matrices + combinations."""
    state = xoshiro_state(cfg.simulation_seed)
    mats, combos = [], []
    for mi, path in enumerate(matrix_paths):
        H = load_matrix(path, cfg.matrix_format)
        rate = 1.0 - H.m / H.n
        qmp = []  # (config_qber, extra fields)
        if cfg.rate_adaptation:
            unt = None
            if cfg.untainted_puncturing:
                unt = _punctured_bits_untainted(path, H, state)
            if cfg.use_adaptation_ranges:
                deltas, effs = _adapt_ranges(cfg, rate)
                pts = [(q, d, e) for q in _rate_qber_values(cfg, rate) for d in deltas for e in effs]
            else:
                pts = _adapt_maps(cfg, rate)
            for q, d, e in pts:
                p, s, ar = adapt_code_rate(H.n, H.m, q, d, e, unt, state)
                if p.size == 0 and s.size == 0:
                    continue  # the reference's "beyond the achievable rate range" skip
                btr = _bits_to_remove(H, p, s) if cfg.enable_privacy_maintenance else p.size + s.size
                qmp.append((q, dict(punctured=p, shortened=s, delta=d, efficiency=e, adapted_rate=ar,
                                    bits_to_remove=btr)))
        else:
            btr = _bits_to_remove(H) if cfg.enable_privacy_maintenance else 0
            qmp = [(q, dict(bits_to_remove=btr)) for q in _rate_qber_values(cfg, rate)]
        if cfg.decoding_algorithm in (2, 3):
            sfs = [(a, 0.0) for a in _factor_values(cfg.primary, rate)]
        elif cfg.decoding_algorithm in (4, 5):
            sfs = [(a, b) for a in _factor_values(cfg.primary, rate) for b in _factor_values(cfg.secondary, rate)]
        else:
            sfs = [(0.0, 0.0)]
        mats.append((path, H))
        for q, extra in qmp:
            for a, b in sfs:
                combos.append(Combination(mi, q, a, b, **extra))
    return mats, combos


# ---- trials on the GPU + statistics -------------------------------------------
def shard_ranges(total: int, shards: int) -> list[tuple[int, int]]:
    """Contiguous trial slices [b, e) of ceil(total / shards) trials, one per
    shard; trailing shards may be short or empty — the
    slices qldpc_run_trials gives the graph's devices (qldpc_shard_range)."""
    import ctypes

    from ._lib import check, lib

    shards = max(1, int(shards))
    out = []
    for k in range(shards):
        lo, hi = ctypes.c_int32(), ctypes.c_int32()
        check(lib().qldpc_shard_range(int(total), shards, k, ctypes.byref(lo), ctypes.byref(hi)), "qldpc_shard_range")
        out.append((lo.value, hi.value))
    return out


def run(cfg: Config, mats, combos, device: int = 0, log=print, devices=None):
    """The simulation loop over combinations (src/simulation.cpp:700-760).

    Each combination's TRIALS_NUMBER trials go through the C ABI's batch seam
    (qldpc_run_trials: the body of the reference's pool.detach_loop over
    run_trial, :721-746): the per-trial seeds in, and per trial
    {iterations_num, syndromes_match, keys_match, runtime} out; keys, frames,
    decode and key comparison all stay on device.  devices: the GPUs the
    trials are sharded over (default [device]) — contiguous slices, one host
    thread and stream pair per entry inside the library, no collective.  An
    entry may repeat a device (several concurrent shards on one GPU).  The
    statistics do not depend on the sharding: every trial's result is a
    function of its seed alone."""
    devs = [int(d) for d in (devices if devices else [device])]
    seeds = trial_seeds(cfg.simulation_seed, cfg.trials_number)
    graphs = {}  # matrix -> Graph replicated on devs
    results = []

    def submit(sim):
        c = combos[sim]
        path, H = mats[c.matrix_index]
        p = Params(cfg.decoding_algorithm, cfg.max_iterations, cfg.threshold_enabled, cfg.threshold, c.primary,
                   c.secondary)
        if c.matrix_index not in graphs:
            graphs[c.matrix_index] = Graph(H, devices=devs)
        g = graphs[c.matrix_index]
        plan = g.rate_plan(c.punctured, c.shortened) if c.punctured is not None else None
        # trial seed = seeds[n] + curr_sim (:743)
        return g.submit_trials(p, c.config_qber, seeds, seed_add=sim, plan=plan)

    def try_submit(sim):  # an error (run_trial's "too small for QBER") is raised at its own turn
        try:
            return submit(sim)
        except Exception as e:  # noqa: BLE001
            return e

    # combination sim + 1 goes onto the GPUs before combination sim is
    # collected, so its generation overlaps the tail of sim's decode
    nxt = try_submit(0) if combos else None
    for sim, c in enumerate(combos):
        job, nxt = nxt, (try_submit(sim + 1) if sim + 1 < len(combos) else None)
        if isinstance(job, Exception):
            raise job
        out = job.wait()
        path, H = mats[c.matrix_index]
        r = _stats(cfg, sim, os.path.basename(path), H, c, out.accurate_qber, out.iterations.astype(np.int64),
                   out.synd_ok.astype(bool), out.keys_match.astype(bool), out.runtime_us)
        results.append(r)
        log(f"[{sim + 1}/{len(combos)}] {r['matrix_filename']} QBER={c.config_qber:.4f} "
            f"FER={1 - r['ratio_success_ldpc']:.4f} iters={r['iter_mean']:.2f}")
    return results


def throughput_stats(out_len: int, runtime_us: np.ndarray, trials_number: int, rtt_ms: float | None = None):
    """THROUGHPUT_MEAN / STD / MIN / MAX of process_trials_results
    (src/simulation.cpp:626-681): per trial out_len / runtime in bits/s (plus
    the RTT when CONSIDER_RTT), mean and population std over TRIALS_NUMBER, each
    truncated to an integer as the reference's size_t fields.  runtime_us: the
    trial_result::runtime of each trial (qldpc_run_trials: its share of its
    chunk's measured window by its own decode span), held — as the reference's
    std::chrono::microseconds field holds it, and as the C++ batch seam
    (simulation_batch.cpp) stores it — in whole microseconds, rounded to
    nearest and at least 1."""
    rt = np.maximum(1.0, np.floor(np.asarray(runtime_us, np.float64) + 0.5))
    denom = rt + (rtt_ms * 1000.0 if rtt_ms is not None else 0.0)
    tp = out_len * 1e6 / denom
    mean = float(tp.sum()) / trials_number
    std = math.sqrt(float(((tp - mean) ** 2).sum()) / trials_number)
    return int(mean), int(std), int(tp.min()), int(tp.max())


def _stats(cfg, sim, fname, H, c, q_acc, it, ok, km, runtime_us) -> dict:
    """process_trials_results (src/simulation.cpp:580-690)."""
    succ = it[ok]
    mean = float(succ.mean()) if succ.size else 0.0
    std = math.sqrt(float(((succ.astype(np.float64) - mean) ** 2).sum()) / succ.size) if succ.size else 0.0
    r = {"sim_number": sim, "matrix_filename": fname, "is_regular": H.is_regular, "n": H.n, "m": H.m,
         "config_qber": c.config_qber, "accurate_qber": q_acc, "iter_mean": mean, "iter_std": std,
         "iter_min": int(succ.min()) if succ.size else 0, "iter_max": int(succ.max()) if succ.size else 0,
         "ratio_success_dec": ok.sum() / cfg.trials_number, "ratio_success_ldpc": (ok & km).sum() / cfg.trials_number,
         "delta": c.delta, "efficiency": c.efficiency,
         "punct_fraction": (c.punctured.size / H.n) if c.punctured is not None else 0.0,
         "short_fraction": (c.shortened.size / H.n) if c.shortened is not None else 0.0,
         "adapted_rate": c.adapted_rate, "primary": c.primary, "secondary": c.secondary}
    if cfg.enable_throughput_measurement:
        out_len = H.n - c.bits_to_remove if (cfg.rate_adaptation or cfg.enable_privacy_maintenance) else H.n
        tp = throughput_stats(out_len, runtime_us, cfg.trials_number, cfg.rtt if cfg.consider_rtt else None)
        r.update(tp_mean=tp[0], tp_std=tp[1], tp_min=tp[2], tp_max=tp[3])
    return r


# ---- results file (write_file, src/simulation.cpp:4-176) ----------------------
def _f(x: float, prec: int | None = None) -> str:
    """fmt with the reference's custom locale: decimal comma, no grouping."""
    s = f"{x:.{prec}f}" if prec is not None else repr(float(x))
    if prec is None and s.endswith(".0"):
        s = s[:-2]  # fmt's shortest form prints 1.0 as "1"
    return s.replace(".", ",")


def results_filename(cfg: Config, duration: str) -> str:
    ra = "OFF" if not cfg.rate_adaptation else ("ON[punct=untainted]" if cfg.untainted_puncturing
                                                 else "ON[punct=random]")
    rtt = f",RTT={cfg.rtt:.3f}ms" if cfg.enable_throughput_measurement and cfg.consider_rtt else ""
    return (f"ldpc(trial_num={cfg.trials_number},dec_alg={DEC_NAMES[cfg.decoding_algorithm]},"
            f"max_dec_alg_iters={cfg.max_iterations},priv_maint={'ON' if cfg.enable_privacy_maintenance else 'OFF'},"
            f"rate_adapt={ra}{rtt},seed={cfg.simulation_seed},sim_duration={duration})")


def write_results(cfg: Config, results: list[dict], duration: str, directory: str) -> str:
    os.makedirs(directory, exist_ok=True)
    base = results_filename(cfg, duration)
    path = os.path.join(directory, base + ".csv")
    k = 1
    while os.path.exists(path):
        path = os.path.join(directory, f"{base}_{k}.csv")
        k += 1
    alg = cfg.decoding_algorithm
    head = ("#;MATRIX_FILENAME;TYPE;R;M;N;CONFIG_QBER;ACCURATE_QBER;ITER_SUCCESS_MEAN;ITER_SUCCESS_STD;"
            "ITER_SUCCESS_MIN;ITER_SUCCESS_MAX;RATIO_SUCCESS_DEC;RATIO_SUCCESS_LDPC;FER")
    if cfg.rate_adaptation:
        head += ";DELTA;EFFICIENCY;PUNCT_FRACTION;SHORT_FRACTION;R_ADAPTED"
    if cfg.enable_throughput_measurement:
        head += ";THROUGHPUT_MEAN;THROUGHPUT_STD;THROUGHPUT_MIN;THROUGHPUT_MAX"
    head += {2: ";ALPHA", 3: ";BETA", 4: ";ALPHA;NU", 5: ";BETA;SIGMA"}.get(alg, "")
    lines = [head]
    for r in results:
        fer = 1.0 - r["ratio_success_ldpc"]
        fer = round(fer * cfg.trials_number) / cfg.trials_number
        line = ";".join([
            str(r["sim_number"]), r["matrix_filename"], "regular" if r["is_regular"] else "irregular",
            _f(1.0 - r["m"] / r["n"], 3), str(r["m"]), str(r["n"]), _f(r["config_qber"], 4),
            _f(r["accurate_qber"], 4), _f(r["iter_mean"], 2), _f(r["iter_std"], 2), str(r["iter_min"]),
            str(r["iter_max"]), _f(r["ratio_success_dec"]), _f(r["ratio_success_ldpc"]), _f(fer)])
        if cfg.rate_adaptation:
            line += ";" + ";".join(_f(r[k], 3) for k in ("delta", "efficiency", "punct_fraction", "short_fraction",
                                                         "adapted_rate"))
        if cfg.enable_throughput_measurement:
            line += ";" + ";".join(str(r[k]) for k in ("tp_mean", "tp_std", "tp_min", "tp_max"))
        if alg >= 2:
            line += ";" + _f(r["primary"], 3)
        if alg >= 4:
            line += ";" + _f(r["secondary"], 3)
        lines.append(line)
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return path


def matrix_files(directory: str) -> list[str]:
    paths = sorted(os.path.join(directory, f) for f in os.listdir(directory) if f.endswith(".mtrx"))
    if not paths:
        raise ConfigError(f"No files with extension '.mtrx' in the directory '{directory}'.")
    return paths


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("configs", nargs="+", help="JSON configuration file(s)")
    ap.add_argument("--matrices", required=True, help="directory of *.mtrx files in the config's matrix_format")
    ap.add_argument("--results", default="results")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--gpus", type=int, default=0,
                    help="shard every combination's trials over GPUs 0..N-1 of this node (0: --device only)")
    a = ap.parse_args(argv)
    devices = list(range(a.gpus)) if a.gpus > 0 else [a.device]
    for i, cp in enumerate(a.configs):
        cfg = Config.load(cp)
        print(f"CONFIG #{i + 1}: {os.path.basename(cp)} — {DEC_NAMES[cfg.decoding_algorithm]}, "
              f"{cfg.trials_number} trials, seed {cfg.simulation_seed}")
        mats, combos = prepare(cfg, matrix_files(a.matrices))
        t0 = time.time()
        res = run(cfg, mats, combos, devices=devices)
        dt = int(time.time() - t0)
        dur = f"{dt // 3600:02d}h-{dt % 3600 // 60:02d}m-{dt % 60:02d}s"
        print("The results are written to the file:", write_results(cfg, res, dur, a.results))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
