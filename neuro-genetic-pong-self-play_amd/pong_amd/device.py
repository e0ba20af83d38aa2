"""Device-resident entry points over ``libpong_ga.so``.

PyTorch is used only to own device memory and streams: every compute call
goes through the C-ABI (``include/pong_ga.h``) with ``data_ptr()`` pointers and
the current HIP stream.  Nothing here computes on the CPU.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional

import torch

from . import _lib as L

PRECISIONS = {"certified": L.PG_PREC_CERTIFIED, "f64": L.PG_PREC_F64}
PREPS = {"all": L.PG_PREP_ALL, "genomes": L.PG_PREP_GENOMES, "rest": L.PG_PREP_REST}
KERNELS = {"auto": L.PG_KERNEL_AUTO, "general": L.PG_KERNEL_GENERAL, "split": L.PG_KERNEL_SPLIT,
           "wide": L.PG_KERNEL_WIDE}
DTYPES = {torch.float32: L.PG_F32, torch.float64: L.PG_F64}


def gene_count(nodes, bias=True) -> int:
    """utils.calculate_gene_size (utils.py:128-136) for an arbitrary shape."""
    b = 1 if bias else 0
    return sum((int(nodes[i]) + b) * int(nodes[i + 1]) for i in range(len(nodes) - 1))


def _ptr(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _need(t: torch.Tensor, name: str, dtype, device, shape=None):
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if t.device != device:
        raise ValueError(f"{name} must live on {device}, got {t.device}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} must have shape {tuple(shape)}, got {tuple(t.shape)}")


def _need_rows(t: torch.Tensor, name: str, dtype, device):
    """A row-major matrix whose rows may be strided (pg_eval_args.opponent_stride):
    e.g. a rank's slice hall[b::K] of the hall of fame."""
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if t.device != device:
        raise ValueError(f"{name} must live on {device}, got {t.device}")
    if t.dim() != 2 or (t.shape[1] > 1 and t.stride(1) != 1) or (t.shape[0] > 1 and t.stride(0) < t.shape[1]):
        raise ValueError(f"{name} must be row-major rows (unit column stride, row stride >= row length)")


@dataclass
class EvalResult:
    """evaluate() outputs for a batch, all on the device."""

    fitness: torch.Tensor       # [n] f64
    rewards: torch.Tensor       # [n, games] f64
    scores: torch.Tensor        # [n, games, 2] int32 (score1, score2)
    frames: torch.Tensor        # [n, games] int32 env steps
    total_frames: torch.Tensor  # [n, games] f64
    status: torch.Tensor        # [n] int32, 1 = ZeroDivisionError
    counters: torch.Tensor      # [16] int64 (pg_eval_args.counters): [0] env steps stepped one frame at
    #                             a time, [1] NN forwards, [2] numpy-order f64 forwards, [3] games,
    #                             [4..6] certificate cascade (split), [7] network passes (wide), [8]
    #                             frames of periodic rallies advanced at once, [12] serve-delay frames
    #                             advanced at once (the episodes' frames = [0] + [8] + [12])


class Evaluator:
    """Population evaluator for one NETWORK_SHAPE on one device."""

    def __init__(self, nodes, bias=True, dtype=torch.float64, device=None, n_games=6,
                 precision="certified", kernel="auto", group_lanes=0, seed=0, horizon=0,
                 timeout_thresh=0, win_score=0):
        if not torch.cuda.is_available():
            raise RuntimeError("pong_amd.Evaluator needs a HIP device (no CPU fallback)")
        L.lib()
        self.nodes = [int(n) for n in nodes]
        self.bias = bool(bias)
        self.dtype = dtype
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.n_games = int(n_games)
        self.precision = precision
        self.kernel = kernel
        self.group_lanes = int(group_lanes)
        self.seed = int(seed)
        # pg_eval_args.horizon: 0 = evaluate()'s episodes; T > 0 = SURVEY 8(d)'s
        # fixed-horizon measurement mode (T frames per game slot, auto-reset)
        self.horizon = int(horizon)
        # pg_eval_args.timeout_thresh / win_score: config.py's TIMEOUT_THRESH and
        # WIN_SCORE (perform_episode's termination, main.py:102-107); 0 = 2000 / 3
        self.timeout_thresh = int(timeout_thresh)
        self.win_score = int(win_score)
        self.genes = gene_count(self.nodes, self.bias)
        self.net = L.make_net(self.nodes, self.bias, DTYPES[dtype])
        self._ws = None
        self._prep_key = self._prep_ws = None  # what the last prep="genomes" call left in the workspace

    # ------------------------------------------------------------ schedules
    def selfplay_schedule(self, n: int, n_opponents: int, offset: int = 0):
        """All games NN vs hall-of-fame row (global_index * games + g) % n_opponents."""
        dev = self.device
        gi = (torch.arange(n, device=dev, dtype=torch.int64) + offset)[:, None] * self.n_games
        gi = gi + torch.arange(self.n_games, device=dev, dtype=torch.int64)[None, :]
        kind = torch.full((n, self.n_games), L.PG_OPP_NN, dtype=torch.int32, device=dev)
        opp = (gi % max(n_opponents, 1)).to(torch.int32)
        mult = torch.ones((n, self.n_games), dtype=torch.float64, device=dev)
        return kind, opp, mult

    # ------------------------------------------------------------- evaluate
    def _workspace(self, args: L.PgEvalArgs) -> torch.Tensor:
        need = L.lib().pg_eval_workspace_bytes(ctypes.byref(args))
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(max(need, 4096), dtype=torch.uint8, device=self.device)
        return self._ws

    def evaluate(self, genomes: torch.Tensor, kind: torch.Tensor, opp: torch.Tensor, mult: torch.Tensor,
                 opponents: Optional[torch.Tensor] = None, trace_games: int = 0, trace_cap: int = 0,
                 out: Optional[EvalResult] = None, precision: Optional[str] = None,
                 kernel: Optional[str] = None, group_lanes: Optional[int] = None, validate: bool = True,
                 hard_log: Optional[torch.Tensor] = None, rows: Optional[torch.Tensor] = None,
                 n_active: Optional[torch.Tensor] = None, prep: str = "all", horizon: Optional[int] = None):
        """Run every genome's games to termination; returns (EvalResult, trace or None).

        ``validate`` checks the schedule's opponent rows on the host first (one
        device sync); callers that built the schedule themselves may skip it.
        ``hard_log`` ([cap, 8] int32, device) receives the decisions no bound
        settles (pg_eval_args.hard_log); ``counters[9]`` counts them.
        ``rows`` ([n] int32, device): evaluate genomes rows ``rows[i]`` (results
        indexed by i) -- eaSimple's ``invalid_ind`` without copying rows.
        ``n_active`` ([1] int32, device): play only entries i < n_active[0]
        (the others' results are left untouched).
        ``prep`` (pg_eval_args.prep): "all"; "genomes" only prepares the split
        kernel's genome records (no games: ``out`` is left untouched); "rest"
        plays after such a call with the same genomes, rows, n_active and
        evaluator (its workspace holds the records), preparing the opponents'
        records first.
        ``horizon`` (pg_eval_args.horizon, default ``self.horizon``): T > 0 runs
        every game slot for exactly T frames with auto-reset (rewards = the
        completed episodes' sum, total_frames = their count; see pong_ga.h).
        Only the split kernel's bench layout has it: [6, 33..64, 3] networks on
        the default 8-lane groups, untraced (else PongGAError).
        """
        dev = self.device
        n = genomes.shape[0] if rows is None else rows.shape[0]
        games = self.n_games
        _need(genomes, "genomes", self.dtype, dev)
        if genomes.dim() != 2 or genomes.shape[1] < self.genes:
            raise ValueError(f"genomes must be [n, >= {self.genes}], got {tuple(genomes.shape)}")
        _need(kind, "kind", torch.int32, dev, (n, games))
        _need(opp, "opp", torch.int32, dev, (n, games))
        _need(mult, "mult", torch.float64, dev, (n, games))
        if opponents is not None:
            _need_rows(opponents, "opponents", self.dtype, dev)
            if opponents.dim() != 2 or opponents.shape[1] < self.genes:
                raise ValueError(f"opponents must be [H, >= {self.genes}], got {tuple(opponents.shape)}")
        if rows is not None:
            _need(rows, "rows", torch.int32, dev, (n,))
        if validate and n:
            # one host sync: out-of-range rows would fault the GPU, so check before launching
            if rows is not None and bool(((rows < 0) | (rows >= genomes.shape[0])).any()):
                raise ValueError(f"rows must index the {genomes.shape[0]}-row genomes tensor")
            nn_games = kind == L.PG_OPP_NN
            if bool(((kind < 0) | (kind > L.PG_OPP_NN)).any()):
                raise ValueError("kind values must be pg_opp_kind codes 0..3")
            if bool(nn_games.any()):
                h = 0 if opponents is None else opponents.shape[0]
                bad = nn_games & ((opp < 0) | (opp >= h))
                if bool(bad.any()):
                    raise ValueError(f"opp rows must index the {h}-row opponents tensor")
        if out is None:
            out = EvalResult(
                fitness=torch.empty(n, dtype=torch.float64, device=dev),
                rewards=torch.empty((n, games), dtype=torch.float64, device=dev),
                scores=torch.empty((n, games, 2), dtype=torch.int32, device=dev),
                frames=torch.empty((n, games), dtype=torch.int32, device=dev),
                total_frames=torch.empty((n, games), dtype=torch.float64, device=dev),
                status=torch.empty(n, dtype=torch.int32, device=dev),
                counters=torch.empty(16, dtype=torch.int64, device=dev))
        # (the counters are zeroed by pg_eval_population itself)
        trace = None
        if trace_games and trace_cap:
            trace = torch.zeros((trace_games, trace_cap), dtype=torch.uint8, device=dev)
        a = L.PgEvalArgs()
        a.net = self.net
        a.n_genomes = n
        a.n_games = games
        a.genomes = _ptr(genomes)
        a.genome_stride = genomes.stride(0) if genomes.shape[0] > 1 else genomes.shape[1]
        a.genome_rows = _ptr(rows)
        if n_active is not None:
            _need(n_active, "n_active", torch.int32, dev, (1,))
            a.n_active = _ptr(n_active)
        if opponents is not None and opponents.shape[0] > 0:
            a.opponents = _ptr(opponents)
            a.opponent_stride = opponents.stride(0) if opponents.shape[0] > 1 else opponents.shape[1]
            a.n_opponents = opponents.shape[0]
        a.precision = PRECISIONS[precision or self.precision]
        a.game_kind, a.game_opp, a.game_mult = _ptr(kind), _ptr(opp), _ptr(mult)
        a.seed = self.seed
        a.fitness, a.rewards, a.scores = _ptr(out.fitness), _ptr(out.rewards), _ptr(out.scores)
        a.frames, a.total_frames, a.status = _ptr(out.frames), _ptr(out.total_frames), _ptr(out.status)
        a.counters = _ptr(out.counters)
        if trace is not None:
            a.trace, a.trace_games, a.trace_cap = _ptr(trace), trace_games, trace_cap
        if hard_log is not None:
            _need(hard_log, "hard_log", torch.int32, dev)
            if hard_log.dim() != 2 or hard_log.shape[1] != 8:
                raise ValueError("hard_log must be [cap, 8] int32")
            a.hard_log, a.hard_cap = _ptr(hard_log), hard_log.shape[0]
        a.prep = PREPS[prep]
        if prep == "rest" and n and self._prep_key != self._prep_of(genomes, rows, n_active, n):
            # pg_eval_args.prep: a "rest" call plays the genome records a "genomes"
            # call left in this evaluator's workspace -- they must be these genomes'
            raise ValueError("prep='rest' needs a preceding prep='genomes' call with the same genomes, rows, "
                             "n_active and row count on this evaluator")
        a.horizon = self.horizon if horizon is None else int(horizon)
        a.timeout_thresh, a.win_score = self.timeout_thresh, self.win_score
        a.kernel = KERNELS[kernel or self.kernel]
        a.group_lanes = self.group_lanes if group_lanes is None else int(group_lanes)
        ws = self._workspace(a)
        a.workspace, a.workspace_bytes = _ptr(ws), ws.numel()
        if prep == "rest" and n and self._prep_ws != ws.data_ptr():
            raise ValueError("prep='rest': the workspace holding the genome records was reallocated")
        with torch.cuda.device(dev):
            L.check("pg_eval_population", L.lib().pg_eval_population(ctypes.byref(a), _stream(dev)))
        # the genome records in the workspace now belong to this call's genomes (or to no one)
        self._prep_key = self._prep_of(genomes, rows, n_active, n) if prep == "genomes" else None
        self._prep_ws = ws.data_ptr() if prep == "genomes" else None
        return out, trace

    @staticmethod
    def _prep_of(genomes, rows, n_active, n):
        return (genomes.data_ptr(), genomes.stride(0), None if rows is None else rows.data_ptr(),
                None if n_active is None else n_active.data_ptr(), int(n))

    # -------------------------------------------------------------- forward
    def forward(self, genomes: torch.Tensor, x: torch.Tensor, genome_index: Optional[torch.Tensor] = None,
                precision: Optional[str] = None, want_act: bool = True, want_layers: bool = False):
        """Batched NeuralNetwork.run: returns (argmax index [n] int32, activations [n, out] f64).

        ``want_layers`` (precision "f64" only) also stores every layer's
        pre-activations and activations in ``self.last_layers`` = (z, h), each
        [n, sum(nodes[1:])] f64.
        """
        dev = self.device
        _need(genomes, "genomes", self.dtype, dev)
        n = x.shape[0]
        _need(x, "x", torch.float64, dev, (n, self.nodes[0]))
        if genome_index is not None:
            _need(genome_index, "genome_index", torch.int32, dev, (n,))
        index = torch.empty(n, dtype=torch.int32, device=dev)
        act = torch.empty((n, self.nodes[-1]), dtype=torch.float64, device=dev) if want_act else None
        counters = torch.zeros(4, dtype=torch.int64, device=dev)
        a = L.PgForwardArgs()
        a.net = self.net
        a.n = n
        a.genomes = _ptr(genomes)
        a.genome_stride = genomes.stride(0) if genomes.shape[0] > 1 else genomes.shape[1]
        a.genome_index = _ptr(genome_index)
        a.x = _ptr(x)
        a.precision = PRECISIONS[precision or self.precision]
        a.index = _ptr(index)
        a.act = _ptr(act)
        a.counters = _ptr(counters)
        if want_layers:
            units = sum(self.nodes[1:])
            z_all = torch.empty((n, units), dtype=torch.float64, device=dev)
            h_all = torch.empty((n, units), dtype=torch.float64, device=dev)
            a.z_all, a.h_all = _ptr(z_all), _ptr(h_all)
            self.last_layers = (z_all, h_all)
        with torch.cuda.device(dev):
            L.check("pg_forward", L.lib().pg_forward(ctypes.byref(a), _stream(dev)))
        self.last_forward_counters = counters
        return index, act

    # --------------------------------------------------------------- decide
    def decide(self, genomes: torch.Tensor, k: torch.Tensor, genome_index: Optional[torch.Tensor] = None):
        """The split kernel's decision cascade (pg_decide) on doubled-centroid
        features k [n, 6] int32: returns (argmax index [n] int32, stage [n] int32):
        0 f32 certificate, 1 in-wave plateau rule, 2 certified f64 rules,
        3 numpy-order f64 forward, 4 the f32 rules under the frame's own bound
        (pg_decide_args.stage)."""
        dev = self.device
        _need(genomes, "genomes", self.dtype, dev)
        n = k.shape[0]
        _need(k, "k", torch.int32, dev, (n, 6))
        if genome_index is not None:
            _need(genome_index, "genome_index", torch.int32, dev, (n,))
        index = torch.empty(n, dtype=torch.int32, device=dev)
        stage = torch.empty(n, dtype=torch.int32, device=dev)
        a = L.PgDecideArgs()
        a.net = self.net
        a.n = n
        a.genomes = _ptr(genomes)
        a.genome_stride = genomes.stride(0) if genomes.shape[0] > 1 else genomes.shape[1]
        a.genome_index = _ptr(genome_index)
        a.k = _ptr(k)
        a.index = _ptr(index)
        a.stage = _ptr(stage)
        with torch.cuda.device(dev):
            L.check("pg_decide", L.lib().pg_decide(ctypes.byref(a), _stream(dev)))
        return index, stage

    def wide_decide(self, genomes: torch.Tensor, k: torch.Tensor, genome_index: Optional[torch.Tensor] = None):
        """k_wide's own decision (pg_wide_decide: one frame of the evaluation
        kernel per pass) on doubled-centroid features k [n, 6] int32: returns
        (argmax index [n] int32, output activations [n, out] f64)."""
        dev = self.device
        _need(genomes, "genomes", self.dtype, dev)
        n = k.shape[0]
        _need(k, "k", torch.int32, dev, (n, 6))
        if genome_index is not None:
            _need(genome_index, "genome_index", torch.int32, dev, (n,))
        index = torch.empty(n, dtype=torch.int32, device=dev)
        act = torch.empty((n, self.nodes[-1]), dtype=torch.float64, device=dev)
        a = L.PgWideDecideArgs()
        a.net = self.net
        a.n = n
        a.genomes = _ptr(genomes)
        a.genome_stride = genomes.stride(0) if genomes.shape[0] > 1 else genomes.shape[1]
        a.genome_index = _ptr(genome_index)
        a.k = _ptr(k)
        a.index = _ptr(index)
        a.act = _ptr(act)
        nbytes = L.lib().pg_wide_decide_workspace_bytes(ctypes.byref(a))
        ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        a.workspace, a.workspace_bytes = _ptr(ws), nbytes
        with torch.cuda.device(dev):
            L.check("pg_wide_decide", L.lib().pg_wide_decide(ctypes.byref(a), _stream(dev)))
        return index, act


class Physics:
    """The SoA Pong stepper (pg_physics_reset / pg_physics_step) for n games."""

    def __init__(self, n: int, device=None):
        L.lib()
        self.n = int(n)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.state = torch.zeros((L.PG_STATE_FIELDS, self.n), dtype=torch.int32, device=self.device)

    def reset(self, seeds: torch.Tensor, one_player: Optional[torch.Tensor] = None):
        _need(seeds, "seeds", torch.int64, self.device, (self.n,))
        if one_player is not None:
            _need(one_player, "one_player", torch.int32, self.device, (self.n,))
        with torch.cuda.device(self.device):
            L.check("pg_physics_reset", L.lib().pg_physics_reset(
                _ptr(self.state), self.n, _ptr(seeds), _ptr(one_player), _stream(self.device)))

    def step(self, actions: torch.Tensor):
        """actions [n] uint8: bit0 right up, bit1 right down, bit2 left up, bit3 left down."""
        _need(actions, "actions", torch.uint8, self.device, (self.n,))
        with torch.cuda.device(self.device):
            L.check("pg_physics_step", L.lib().pg_physics_step(
                _ptr(self.state), self.n, _ptr(actions), _stream(self.device)))

    def fields(self) -> dict:
        s = self.state.cpu()
        return {name: s[i] for i, name in enumerate(L.STATE_FIELD_NAMES)}


def select_tournament(fitness: torch.Tensor, k: int, tournsize: int, seed: int, generation: int) -> torch.Tensor:
    """tools.selTournament on device: returns [k] int32 rows of the winners."""
    _need(fitness, "fitness", torch.float64, fitness.device)
    chosen = torch.empty(k, dtype=torch.int32, device=fitness.device)
    a = L.PgSelectArgs(fitness.shape[0], k, tournsize, _ptr(fitness), _ptr(chosen), seed, generation)
    with torch.cuda.device(fitness.device):
        L.check("pg_ga_select_tournament", L.lib().pg_ga_select_tournament(ctypes.byref(a), _stream(fitness.device)))
    return chosen


def select_tournament_ranked(fitness: torch.Tensor, k: int, tournsize: int, seed: int, generation: int) -> torch.Tensor:
    """tools.selTournament's winner distribution by rank sampling (O(n log n), any tournsize)."""
    _need(fitness, "fitness", torch.float64, fitness.device)
    sorted_fit, order = torch.sort(fitness, stable=True)
    order = order.to(torch.int32)
    chosen = torch.empty(k, dtype=torch.int32, device=fitness.device)
    a = L.PgSelectArgs(fitness.shape[0], k, tournsize, _ptr(fitness), _ptr(chosen), seed, generation)
    with torch.cuda.device(fitness.device):
        L.check("pg_ga_select_tournament_ranked", L.lib().pg_ga_select_tournament_ranked(
            ctypes.byref(a), _ptr(sorted_fit), _ptr(order), _stream(fitness.device)))
    return chosen


def vary(parents: torch.Tensor, chosen: torch.Tensor, genes: int, cxpb: float, mutpb: float, alpha: float,
         mu: float, sigma: float, indpb: float, seed: int, generation: int, out: Optional[torch.Tensor] = None,
         pair_mask: Optional[torch.Tensor] = None, invalid: Optional[torch.Tensor] = None,
         pair_list: Optional[tuple] = None):
    """algorithms.varAnd(cxBlend, mutGaussian) on device: returns (offspring, invalid[n] uint8).
    ``pair_mask`` ([(n + 1) // 2] uint8): only the marked pairs' rows are
    written (the invalid flags of every row are); see pg_ga_args.pair_mask."""
    dev = parents.device
    n = chosen.shape[0]
    _need(chosen, "chosen", torch.int32, dev, (n,))
    if pair_mask is not None:
        _need(pair_mask, "pair_mask", torch.uint8, dev, ((n + 1) // 2,))
    if out is None:
        out = torch.empty((n, parents.shape[1]), dtype=parents.dtype, device=dev)
    if invalid is None:
        invalid = torch.empty(n, dtype=torch.uint8, device=dev)
    _need(invalid, "invalid", torch.uint8, dev, (n,))
    a = L.PgGaArgs()
    a.n, a.genes, a.dtype = n, genes, DTYPES[parents.dtype]
    a.parents, a.stride, a.n_parents = _ptr(parents), parents.stride(0), parents.shape[0]
    a.chosen, a.offspring, a.invalid = _ptr(chosen), _ptr(out), _ptr(invalid)
    a.cxpb, a.mutpb, a.alpha, a.mu, a.sigma, a.indpb = cxpb, mutpb, alpha, mu, sigma, indpb
    a.seed, a.generation = seed, generation
    a.pair_mask = _ptr(pair_mask)
    if pair_list is not None:  # (list [cap] int32, count [1] int32, cap): only the listed pairs
        lst, cnt, cap = pair_list
        _need(lst, "pair_list", torch.int32, dev)
        _need(cnt, "pair_count", torch.int32, dev, (1,))
        a.pair_list, a.pair_count, a.pair_cap = _ptr(lst), _ptr(cnt), int(min(cap, lst.numel()))
    if out.stride(0) != parents.stride(0):
        raise ValueError("offspring and parents must share the row stride")
    with torch.cuda.device(dev):
        L.check("pg_ga_vary", L.lib().pg_ga_vary(ctypes.byref(a), _stream(dev)))
    return out, invalid


def list_pairs(mask: torch.Tensor, out: torch.Tensor, count: torch.Tensor) -> None:
    """pg_ga_list_pairs: out[:count] = the marked pairs (any order)."""
    dev = mask.device
    _need(mask, "pair_mask", torch.uint8, dev)
    _need(out, "pair_list", torch.int32, dev)
    _need(count, "pair_count", torch.int32, dev, (1,))
    if out.numel() < mask.numel():
        raise ValueError("pair_list must hold every pair")
    with torch.cuda.device(dev):
        L.check("pg_ga_list_pairs", L.lib().pg_ga_list_pairs(_ptr(mask), mask.numel(), _ptr(out), _ptr(count),
                                                             _stream(dev)))


def mark_pairs(mask: torch.Tensor, rows: torch.Tensor, skip: tuple = (0, 0),
               exclude: Optional[torch.Tensor] = None) -> None:
    """pg_ga_mark_pairs: mask[rows >> 1] = 1 except the pairs in [skip[0],
    skip[1]) and those ``exclude`` marks."""
    dev = mask.device
    _need(mask, "pair_mask", torch.uint8, dev)
    _need(rows, "rows", torch.int32, dev)
    if exclude is not None:
        _need(exclude, "exclude", torch.uint8, dev, tuple(mask.shape))
    with torch.cuda.device(dev):
        L.check("pg_ga_mark_pairs", L.lib().pg_ga_mark_pairs(_ptr(mask), mask.shape[0], _ptr(rows), rows.numel(),
                                                             int(skip[0]), int(skip[1]), _ptr(exclude), _stream(dev)))


SCHEDULES = {"reference": L.PG_SCHED_REFERENCE, "selfplay": L.PG_SCHED_SELFPLAY}


def schedule(mode: str, n: int, n_games: int, row_offset: int, hof_fitness: Optional[torch.Tensor], n_hof: int,
             seed: int, generation: int, device, rows: Optional[torch.Tensor] = None, hof_slices: int = 1,
             block_rows: int = 0, slice_local: bool = False, out: Optional[tuple] = None):
    """pg_ga_schedule: (kind, opp, mult) [n, n_games] of evaluate()'s games on device
    (``out``: the three tensors to write, else fresh ones);
    ``rows`` ([n] int32) gives entry i's global population row (default row_offset + i).
    Self-play with ``hof_slices`` K > 1: the genomes of row block r // block_rows
    play the hall's interleaved slice (r // block_rows) mod K (pong_ga.h); with
    ``slice_local`` opp indexes the slice (pass ``hall[b::K]`` as the opponents)."""
    dev = torch.device(device)
    if out is None:
        kind = torch.empty((n, n_games), dtype=torch.int32, device=dev)
        opp = torch.empty((n, n_games), dtype=torch.int32, device=dev)
        mult = torch.empty((n, n_games), dtype=torch.float64, device=dev)
    else:
        kind, opp, mult = out
        _need(kind, "kind", torch.int32, dev, (n, n_games))
        _need(opp, "opp", torch.int32, dev, (n, n_games))
        _need(mult, "mult", torch.float64, dev, (n, n_games))
    if hof_fitness is not None:
        _need(hof_fitness, "hof_fitness", torch.float64, dev)
        if hof_fitness.numel() < n_hof:
            raise ValueError(f"hof_fitness holds {hof_fitness.numel()} values, n_hof={n_hof}")
    elif n_hof and mode == "reference":
        raise ValueError("reference schedule with a hall of fame needs hof_fitness")
    if rows is not None:
        _need(rows, "rows", torch.int32, dev, (n,))
    a = L.PgScheduleArgs(SCHEDULES[mode], n, n_games, row_offset, n_hof, _ptr(hof_fitness), seed, generation,
                         _ptr(kind), _ptr(opp), _ptr(mult), _ptr(rows), int(hof_slices), int(block_rows),
                         1 if slice_local else 0)
    with torch.cuda.device(dev):
        L.check("pg_ga_schedule", L.lib().pg_ga_schedule(ctypes.byref(a), _stream(dev)))
    return kind, opp, mult


def row_hash(rows: torch.Tensor, genes: Optional[int] = None, index: Optional[torch.Tensor] = None) -> torch.Tensor:
    """pg_row_hash: int64 (the uint64 bits) content hash of each row's first
    ``genes`` genes, for every row or for the rows ``index`` names."""
    if rows.dim() != 2 or rows.dtype not in DTYPES or rows.stride(1) != 1:
        raise ValueError("rows must be a row-major [n, G] f32/f64 tensor")
    genes = rows.shape[1] if genes is None else int(genes)
    n = rows.shape[0] if index is None else index.shape[0]
    if index is not None:
        _need(index, "index", torch.int32, rows.device, (n,))
    out = torch.empty(n, dtype=torch.int64, device=rows.device)
    stride = rows.stride(0) if rows.shape[0] > 1 else rows.shape[1]
    with torch.cuda.device(rows.device):
        L.check("pg_row_hash", L.lib().pg_row_hash(_ptr(rows), stride, _ptr(index), n, genes, DTYPES[rows.dtype],
                                                   _ptr(out), _stream(rows.device)))
    return out


def gather_rows(dst: torch.Tensor, old_rows: torch.Tensor, rows: torch.Tensor, src: torch.Tensor, n_old: int,
                index: Optional[torch.Tensor] = None, genes: Optional[int] = None) -> torch.Tensor:
    """pg_gather_rows: dst[j] = old_rows[src[j]] if src[j] < n_old else
    rows[index[src[j] - n_old]] (rows[src[j] - n_old] without index)."""
    dev = dst.device
    n = src.shape[0]
    _need(src, "src", torch.int32, dev, (n,))
    if index is not None:
        _need(index, "index", torch.int64, dev, (index.shape[0],))
    for name, t in (("dst", dst), ("old_rows", old_rows), ("rows", rows)):
        if t.dim() != 2 or t.dtype != dst.dtype or t.device != dev or t.stride(1) != 1:
            raise ValueError(f"{name} must be a row-major [n, G] tensor of dst's dtype on dst's device")
    genes = dst.shape[1] if genes is None else int(genes)
    if n > dst.shape[0]:
        raise ValueError("more source indices than destination rows")
    with torch.cuda.device(dev):
        L.check("pg_gather_rows", L.lib().pg_gather_rows(
            _ptr(dst), dst.stride(0), _ptr(old_rows), old_rows.stride(0), _ptr(rows), rows.stride(0), _ptr(index),
            _ptr(src), int(n_old), n, genes, DTYPES[dst.dtype], _stream(dev)))
    return dst


def hof_rank_classes(hof_fitness: torch.Tensor, hof_hash: torch.Tensor, cand_fitness: torch.Tensor,
                     cand_hash: torch.Tensor) -> torch.Tensor:
    """pg_hof_rank_classes: the packed scan input of HallOfFame.update on the
    device -- int64 [n + k] (n = members + k candidates): rank | class << 32 per
    entry (members in items order first), then the candidates' fitness bits."""
    dev = cand_fitness.device
    hn, k = hof_fitness.shape[0], cand_fitness.shape[0]
    _need(hof_fitness, "hof_fitness", torch.float64, dev, (hn,))
    _need(hof_hash, "hof_hash", torch.int64, dev, (hn,))
    _need(cand_fitness, "cand_fitness", torch.float64, dev, (k,))
    _need(cand_hash, "cand_hash", torch.int64, dev, (k,))
    packed = torch.empty(hn + 2 * k, dtype=torch.int64, device=dev)
    nbytes = int(L.lib().pg_hof_rank_classes_workspace_bytes(hn + k))
    if nbytes == 0:
        msg = L.lib().pg_last_error()
        raise L.PongGAError("pg_hof_rank_classes_workspace_bytes", -1, msg.decode() if msg else "")
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    a = L.PgHofRankArgs(hn, _ptr(hof_fitness), _ptr(hof_hash), k, _ptr(cand_fitness), _ptr(cand_hash),
                        _ptr(packed), _ptr(ws), nbytes)
    with torch.cuda.device(dev):
        L.check("pg_hof_rank_classes", L.lib().pg_hof_rank_classes(ctypes.byref(a), _stream(dev)))
    return packed


def hof_prepare(fitness: torch.Tensor, worst: Optional[float], rows: torch.Tensor, genes: int,
                hof_fitness: torch.Tensor, hof_hash: torch.Tensor):
    """pg_hof_prepare: the device half of HallOfFame.update in one call.
    Candidates are every row (worst None) or the rows with fitness > worst.
    Returns (k, cand [k] int64 rows, hashes [hof_n + k] int64, packed
    [hof_n + 2k] int64 as hof_rank_classes); one host sync (k)."""
    dev = fitness.device
    pn, hn = fitness.shape[0], hof_fitness.shape[0]
    _need(fitness, "fitness", torch.float64, dev, (pn,))
    _need(hof_fitness, "hof_fitness", torch.float64, dev, (hn,))
    _need(hof_hash, "hof_hash", torch.int64, dev, (hn,))
    if rows.dim() != 2 or rows.shape[0] != pn or rows.dtype not in DTYPES or rows.stride(1) != 1 or rows.device != dev:
        raise ValueError("rows must be a row-major [pop_n, G] f32/f64 tensor on fitness's device")
    cand = torch.empty(pn, dtype=torch.int64, device=dev)
    hashes = torch.empty(hn + pn, dtype=torch.int64, device=dev)
    packed = torch.empty(hn + 2 * pn, dtype=torch.int64, device=dev)
    nbytes = int(L.lib().pg_hof_prepare_workspace_bytes(hn, pn))
    if nbytes == 0:
        msg = L.lib().pg_last_error()
        raise L.PongGAError("pg_hof_prepare_workspace_bytes", -1, msg.decode() if msg else "")
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    k = ctypes.c_int32(0)
    stride = rows.stride(0) if pn > 1 else rows.shape[1]
    a = L.PgHofPrepareArgs(_ptr(fitness), pn, 0 if worst is None else 1, 0.0 if worst is None else float(worst),
                           _ptr(rows), stride, int(genes), DTYPES[rows.dtype], hn, _ptr(hof_fitness), _ptr(hof_hash),
                           ctypes.addressof(k), _ptr(cand), _ptr(hashes), _ptr(packed), _ptr(ws), nbytes)
    with torch.cuda.device(dev):
        L.check("pg_hof_prepare", L.lib().pg_hof_prepare(ctypes.byref(a), _stream(dev)))
    k = k.value
    return k, cand[:k], hashes[: hn + k], packed[: hn + 2 * k]


def hof_update(maxsize: int, hof_fitness, hof_hash, pop_fitness, pop_hash, rank=None):
    """pg_hof_update (host, no GPU): HallOfFame.update over fitness/hash arrays.

    ``rank`` (optional, [len(hof) + len(pop)] int32): the entries' positions in
    ascending (fitness, age) order (see pg_hof_args.rank); computed here if None.
    Returns (src [new_n] int32, fitness [new_n] f64): member j comes from old
    member src[j] if src[j] < len(hof_fitness), else from population entry
    src[j] - len(hof_fitness)."""
    import numpy as np
    hf = np.ascontiguousarray(hof_fitness, dtype=np.float64)
    hh = np.ascontiguousarray(np.asarray(hof_hash, dtype=np.int64)).view(np.uint64)
    pf = np.ascontiguousarray(pop_fitness, dtype=np.float64)
    ph = np.ascontiguousarray(np.asarray(pop_hash, dtype=np.int64)).view(np.uint64)
    if hf.shape != hh.shape or pf.shape != ph.shape:
        raise ValueError("fitness and hash arrays must pair up")
    rk = None
    if rank is not None:
        rk = np.ascontiguousarray(rank, dtype=np.int32)
        if rk.shape != (hf.shape[0] + pf.shape[0],):
            raise ValueError("rank must hold one entry per member and population row")
    src = np.zeros(max(maxsize, 1), dtype=np.int32)
    fit = np.zeros(max(maxsize, 1), dtype=np.float64)
    new_n = ctypes.c_int32(0)
    a = L.PgHofArgs(maxsize, hf.shape[0], hf.ctypes.data, hh.ctypes.data, pf.shape[0], pf.ctypes.data,
                    ph.ctypes.data, rk.ctypes.data if rk is not None else None, ctypes.addressof(new_n),
                    src.ctypes.data, fit.ctypes.data)
    L.check("pg_hof_update", L.lib().pg_hof_update(ctypes.byref(a)))
    return src[: new_n.value].copy(), fit[: new_n.value].copy()


def hof_update_packed(maxsize: int, hof_fitness, packed, k: int, slot_in=None, slots: bool = False, out=None):
    """pg_hof_update_packed (host, no GPU): HallOfFame.update from the device's
    packing (pg_hof_prepare_cand: rank | class << 32 per member then per
    candidate, then the candidates' fitness bits); returns (src, fitness) as
    hof_update does, and with ``slots`` the new members' storage slots too
    (the hall in place, ABI 12: ``slot_in`` the current members' slots, None
    = identity).  ``out``: optional int32 numpy array of >= 4 * maxsize
    entries (e.g. a pinned buffer's view) that receives fitness (as f64 in its
    first 2 * maxsize), src and slots back to back -- ready for one upload."""
    import numpy as np
    hf = np.ascontiguousarray(hof_fitness, dtype=np.float64)
    pk = np.ascontiguousarray(packed, dtype=np.int64)
    if pk.shape[0] < hf.shape[0] + 2 * k:
        raise ValueError("packed must hold hof_n + 2k entries")
    M = max(maxsize, 1)
    if out is not None:
        if out.dtype != np.int32 or out.ndim != 1 or out.shape[0] < 4 * M or not out.flags.c_contiguous:
            raise ValueError("out must be a contiguous int32 array of >= 4 * maxsize entries")
        fit, src, slot = out[: 2 * M].view(np.float64), out[2 * M:3 * M], out[3 * M:4 * M]
    else:
        src = np.empty(M, dtype=np.int32)
        fit = np.empty(M, dtype=np.float64)
        slot = np.empty(M, dtype=np.int32)
    sin = None
    if slot_in is not None:
        sin = np.ascontiguousarray(slot_in, dtype=np.int32)
        if sin.shape[0] < hf.shape[0]:
            raise ValueError("slot_in must hold hof_n entries")
    new_n = ctypes.c_int32(0)
    a = L.PgHofPackedArgs(maxsize, hf.shape[0], hf.ctypes.data, int(k), pk.ctypes.data, ctypes.addressof(new_n),
                          src.ctypes.data, fit.ctypes.data, sin.ctypes.data if sin is not None else None,
                          slot.ctypes.data if slots else None)
    L.check("pg_hof_update_packed", L.lib().pg_hof_update_packed(ctypes.byref(a)))
    n = new_n.value
    if slots:
        return src[:n], fit[:n], slot[:n]
    return src[:n], fit[:n]


FRAME_SHAPE = (210, 160, 3)  # obs.npy


def render_frames(state: torch.Tensor, n: Optional[int] = None) -> torch.Tensor:
    """pg_render_frames: [n, 210, 160, 3] uint8 frames of the SoA game states."""
    n = state.shape[1] if n is None else int(n)
    _need(state, "state", torch.int32, state.device, (L.PG_STATE_FIELDS, n))
    frames = torch.empty((n,) + FRAME_SHAPE, dtype=torch.uint8, device=state.device)
    with torch.cuda.device(state.device):
        L.check("pg_render_frames", L.lib().pg_render_frames(_ptr(state), n, _ptr(frames), _stream(state.device)))
    return frames


def find_stuff(frames: torch.Tensor) -> torch.Tensor:
    """pg_find_stuff: [n, 3, 2] f64 centroids (ball, left, right) of [n, 210, 160, 3]
    uint8 frames, NaN where find_stuff returns None."""
    if frames.dim() == 3:
        frames = frames[None]
    if frames.dtype != torch.uint8 or tuple(frames.shape[1:]) != FRAME_SHAPE or not frames.is_contiguous():
        raise ValueError("frames must be contiguous uint8 [n, 210, 160, 3]")
    if frames.data_ptr() % 16:
        frames = frames.clone()
    n = frames.shape[0]
    out = torch.empty((n, 3, 2), dtype=torch.float64, device=frames.device)
    with torch.cuda.device(frames.device):
        L.check("pg_find_stuff", L.lib().pg_find_stuff(_ptr(frames), frames[0].numel() if n else 100800, n, _ptr(out),
                                                       _stream(frames.device)))
    return out


# ------------------------------------------------ one generation's device work
class Workspaces:
    """Grow-only device scratch buffers by name (the C-ABI keeps no allocations)."""

    def __init__(self, device):
        self.device = torch.device(device)
        self._bufs = {}

    def get(self, name: str, nbytes: int) -> torch.Tensor:
        b = self._bufs.get(name)
        if b is None or b.numel() < nbytes:
            b = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=self.device)
            self._bufs[name] = b
        return b

    def tensor(self, name: str, shape, dtype) -> torch.Tensor:
        """A typed view of buffer ``name`` with at least ``shape`` elements."""
        n = 1
        for s in (shape if isinstance(shape, (tuple, list)) else (shape,)):
            n *= int(s)
        item = torch.empty((), dtype=dtype).element_size()
        return self.get(name, n * item)[: n * item].view(dtype).view(shape)


def scatter_fitness(res: EvalResult, n: int, row_lo: int, rows: Optional[torch.Tensor], count: Optional[torch.Tensor],
                    shard_fitness: torch.Tensor, lineage: Optional[torch.Tensor]) -> torch.Tensor:
    """pg_ga_scatter_fitness: the evaluation's fitness in shard row order (rows
    not played read 0) and each played row's longest game into ``lineage``."""
    dev = shard_fitness.device
    _need(shard_fitness, "shard_fitness", torch.float64, dev, (n,))
    if lineage is not None:
        _need(lineage, "lineage", torch.float32, dev)
    games = res.frames.shape[1] if res.frames.dim() == 2 else 1
    a = L.PgScatterArgs(n, games, row_lo, _ptr(res.fitness), _ptr(res.frames), _ptr(rows), _ptr(count),
                        _ptr(shard_fitness), _ptr(lineage))
    with torch.cuda.device(dev):
        L.check("pg_ga_scatter_fitness", L.lib().pg_ga_scatter_fitness(ctypes.byref(a), _stream(dev)))
    return shard_fitness


def merge_fitness(fitness: torch.Tensor, invalid: Optional[torch.Tensor], inherited: Optional[torch.Tensor],
                  new_fitness: torch.Tensor, worst: Optional[float], cand: torch.Tensor, cand_fitness: torch.Tensor,
                  summary: torch.Tensor, ws: Workspaces) -> None:
    """pg_ga_merge_fitness (see pong_ga.h): new fitness, logbook summary, candidates."""
    dev = fitness.device
    n = fitness.shape[0]
    _need(fitness, "fitness", torch.float64, dev, (n,))
    _need(new_fitness, "new_fitness", torch.float64, dev, (n,))
    _need(cand, "cand", torch.int32, dev, (n,))
    _need(cand_fitness, "cand_fitness", torch.float64, dev, (n,))
    _need(summary, "summary", torch.float64, dev, (8,))
    if invalid is not None:
        _need(invalid, "invalid", torch.uint8, dev, (n,))
        _need(inherited, "inherited", torch.float64, dev, (n,))
    nbytes = int(L.lib().pg_ga_merge_workspace_bytes(n))
    w = ws.get("merge", nbytes)
    a = L.PgMergeArgs(n, _ptr(fitness), _ptr(invalid), _ptr(inherited), _ptr(new_fitness),
                      0 if worst is None else 1, 0.0 if worst is None else float(worst), _ptr(cand),
                      _ptr(cand_fitness), _ptr(summary), _ptr(w), w.numel())
    with torch.cuda.device(dev):
        L.check("pg_ga_merge_fitness", L.lib().pg_ga_merge_fitness(ctypes.byref(a), _stream(dev)))


def select_ranked(fitness: torch.Tensor, k: int, tournsize: int, seed: int, generation: int, ws: Workspaces,
                  chosen: Optional[torch.Tensor] = None) -> torch.Tensor:
    """pg_ga_select_ranked: select_tournament_ranked with the sort inside, one call."""
    dev = fitness.device
    _need(fitness, "fitness", torch.float64, dev)
    if chosen is None:
        chosen = torch.empty(k, dtype=torch.int32, device=dev)
    nbytes = int(L.lib().pg_ga_select_workspace_bytes(fitness.shape[0]))
    w = ws.get("select", nbytes)
    a = L.PgSelectArgs(fitness.shape[0], k, tournsize, _ptr(fitness), _ptr(chosen), seed, generation)
    with torch.cuda.device(dev):
        L.check("pg_ga_select_ranked", L.lib().pg_ga_select_ranked(ctypes.byref(a), _ptr(w), w.numel(), _stream(dev)))
    return chosen


def inherit(chosen: torch.Tensor, fitness: torch.Tensor, inherited: torch.Tensor, lineage_in: torch.Tensor,
            lineage_out: torch.Tensor) -> None:
    """pg_ga_inherit: inherited = fitness[chosen], lineage_out = lineage_in[chosen]."""
    dev = chosen.device
    n = chosen.shape[0]
    _need(chosen, "chosen", torch.int32, dev, (n,))
    _need(inherited, "inherited", torch.float64, dev, (n,))
    _need(lineage_out, "lineage_out", torch.float32, dev, (n,))
    with torch.cuda.device(dev):
        L.check("pg_ga_inherit", L.lib().pg_ga_inherit(_ptr(chosen), n, _ptr(fitness), _ptr(inherited),
                                                       _ptr(lineage_in), _ptr(lineage_out), _stream(dev)))


def order(n: int, row_lo: int, invalid: Optional[torch.Tensor], lineage: Optional[torch.Tensor], by_length: bool,
          rows: torch.Tensor, count: torch.Tensor, ws: Workspaces) -> None:
    """pg_ga_order: the shard's evaluation order (invalid rows first, longest lineage first)."""
    dev = rows.device
    _need(rows, "rows", torch.int32, dev, (n,))
    _need(count, "count", torch.int32, dev, (1,))
    nbytes = int(L.lib().pg_ga_order_workspace_bytes(n))
    w = ws.get("order", nbytes)
    with torch.cuda.device(dev):
        L.check("pg_ga_order", L.lib().pg_ga_order(n, row_lo, _ptr(invalid), _ptr(lineage), 1 if by_length else 0,
                                                   _ptr(rows), _ptr(count), _ptr(w), w.numel(), _stream(dev)))


def hof_prepare_cand(hof_fitness: torch.Tensor, hof_hash: torch.Tensor, cand: torch.Tensor,
                     cand_fitness: torch.Tensor, rows: torch.Tensor, genes: int, cand_hash: torch.Tensor,
                     packed: torch.Tensor, ws: Workspaces) -> None:
    """pg_hof_prepare_cand: hashes of the k candidates and the scan's packed input."""
    dev = cand.device
    hn, k = hof_fitness.shape[0], cand.shape[0]
    _need(hof_fitness, "hof_fitness", torch.float64, dev, (hn,))
    _need(hof_hash, "hof_hash", torch.int64, dev, (hn,))
    _need(cand, "cand", torch.int32, dev, (k,))
    _need(cand_fitness, "cand_fitness", torch.float64, dev, (k,))
    _need(cand_hash, "cand_hash", torch.int64, dev, (k,))
    _need(packed, "packed", torch.int64, dev, (hn + 2 * k,))
    if rows.dim() != 2 or rows.dtype not in DTYPES or rows.stride(1) != 1 or rows.device != dev:
        raise ValueError("rows must be a row-major [n, G] f32/f64 tensor on the candidates' device")
    nbytes = int(L.lib().pg_hof_prepare_cand_workspace_bytes(hn, k))
    if nbytes == 0:
        msg = L.lib().pg_last_error()
        raise L.PongGAError("pg_hof_prepare_cand_workspace_bytes", -1, msg.decode() if msg else "")
    w = ws.get("hof_cand", nbytes)
    stride = rows.stride(0) if rows.shape[0] > 1 else rows.shape[1]
    a = L.PgHofCandArgs(hn, _ptr(hof_fitness), _ptr(hof_hash), k, _ptr(cand), _ptr(cand_fitness), _ptr(rows), stride,
                        int(genes), DTYPES[rows.dtype], _ptr(cand_hash), _ptr(packed), _ptr(w), w.numel())
    with torch.cuda.device(dev):
        L.check("pg_hof_prepare_cand", L.lib().pg_hof_prepare_cand(ctypes.byref(a), _stream(dev)))


def hof_commit(dst: torch.Tensor, old_rows: Optional[torch.Tensor], rows: torch.Tensor, cand: torch.Tensor,
               src: torch.Tensor, n_old: int, genes: int, old_hash: torch.Tensor, cand_hash: torch.Tensor,
               new_hash: torch.Tensor, fitness_in: torch.Tensor, new_fitness: torch.Tensor,
               dst_slot: Optional[torch.Tensor] = None) -> None:
    """pg_hof_commit: the new members' rows, hashes and fitness in one pass;
    with ``dst_slot`` (ABI 12) the hall in place: ``dst`` is the hall's
    storage, member j's row is dst[dst_slot[j]], and only entering
    candidates' rows are written (``old_rows`` unused, may be None)."""
    dev = dst.device
    m = src.shape[0]
    _need(src, "src", torch.int32, dev, (m,))
    _need(fitness_in, "fitness_in", torch.float64, dev, (m,))
    if dst_slot is not None:
        _need(dst_slot, "dst_slot", torch.int32, dev, (m,))
        old_rows = None
    elif old_rows is None:
        raise ValueError("old_rows is required without dst_slot")
    for name, t in (("dst", dst), ("old_rows", old_rows), ("rows", rows)):
        if t is None:
            continue
        if t.dim() != 2 or t.dtype != dst.dtype or t.device != dev or t.stride(1) != 1:
            raise ValueError(f"{name} must be a row-major [n, G] tensor of dst's dtype on dst's device")
    if m > dst.shape[0] or m > new_hash.shape[0] or m > new_fitness.shape[0]:
        raise ValueError("more members than destination rows")
    a = L.PgHofCommitArgs(_ptr(dst), dst.stride(0), _ptr(old_rows) if old_rows is not None else None,
                          old_rows.stride(0) if old_rows is not None else 0, _ptr(rows), rows.stride(0),
                          _ptr(cand), _ptr(src), int(n_old), m, int(genes), DTYPES[dst.dtype], _ptr(old_hash),
                          _ptr(cand_hash), _ptr(new_hash), _ptr(fitness_in), _ptr(new_fitness),
                          _ptr(dst_slot) if dst_slot is not None else None)
    with torch.cuda.device(dev):
        L.check("pg_hof_commit", L.lib().pg_hof_commit(ctypes.byref(a), _stream(dev)))
