"""Device-resident eaSimple: the reference's GA loop (main.py:157-173, which
runs DEAP's ``algorithms.eaSimple`` with the operators ga.py:76-94 registers)
with every per-individual step on the MI355X.

One generation (eaSimple, gen >= 1):

====================================================  =========================================
offspring = varAnd(selTournament(pop, len(pop)))      pg_ga_select_tournament_ranked + pg_ga_vary
evaluate the invalid offspring (evaluate, main.py:28)  pg_ga_schedule + pg_eval_population
halloffame.update(offspring)                           pg_row_hash (device) + pg_hof_update (host)
population[:] = offspring; record avg/std/min/max      main.py:158-162 statistics
====================================================  =========================================

Generation 0 evaluates the initial population and fills the hall of fame.

Storage: one ``[H + P, G]`` buffer, hall-of-fame rows first, and a spare of
the same shape that the next generation is written into, so neither the
variation nor the hall-of-fame gather reads what it writes.  The fused path
keeps the hall IN PLACE (``in_place_hall``, ABI 12): its rows stay in the
first buffer's H rows, member j (items order) in slot ``hof_slot[j]``; an
update writes only the entering candidates' rows, into the slots of the
members they evict (pg_hof_update_packed's slot_out, pg_hof_commit's
dst_slot), where the dense form rewrote all H rows into the spare buffer.
Games index hall positions (the schedule); the evaluation maps them to slots
(or, with a sliced hall, gathers the rank's slice, H/N rows).  The GA state is
replicated on every rank; rank r evaluates rows ``shard_range(P, r, N)`` and
the fitness vector is all-gathered once per generation -- the only collective.

Sharded variation (``shard_vary``, on when N > 1): a rank writes only the
offspring rows it needs -- its shard's before the evaluation, then, once the
all-gathered fitness names them, the hall-of-fame candidates and the parents
the next selection picks (tournaments of P/4 draws pick the top rows and their
tied clones: 5 242 distinct of 524 288 in tools/scale_model.py, nearly all of
them candidates too).  Every offspring row is a pure function of its pair's parent
rows and the (seed, generation) keys (pg_ga_args.pair_mask), so these rows
equal a full varAnd's and the replicated state stays identical across ranks;
the other rows of ``population`` are not current on this rank
(``population_full()`` all-gathers the shards).

Differences from DEAP (DESIGN.md "GA"): random draws are counter-based
(distribution parity, not Mersenne-Twister stream parity); ``similar`` is the
equality of 64-bit gene hashes; only the invalid offspring are evaluated
(``invalid_ind``): unmodified ones keep their parent's fitness as DEAP's
clones do, and their games are not played.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from . import device as D
from . import dist as PD

STAT_FIELDS = ("avg", "std", "min", "max")  # main.py:159-162


class DeviceGA:
    """eaSimple state on one device (one per rank): population, fitness, hall of fame, logbook."""

    def __init__(self, nodes, population_size: int, hof_size: Optional[int] = None,
                 tournsize: Optional[int] = None, *, bias: bool = True, dtype=torch.float64, device=None,
                 n_games: int = 6, schedule: str = "reference", cxpb: float = 0.9, mutpb: float = 0.9,
                 alpha: float = 0.9, mu: float = 0.0, sigma: float = 0.9, indpb: float = 0.9,
                 seed: int = 0, physics_seed: int = 0, precision: str = "certified", kernel: str = "auto",
                 group=None, hof_block_rows: int = 0, timeout_thresh: int = 0, win_score: int = 0):
        if schedule not in D.SCHEDULES:
            raise ValueError(f"schedule must be one of {sorted(D.SCHEDULES)}")
        self.nodes = [int(v) for v in nodes]
        self.P = int(population_size)
        # HALL_OF_FAME_AMOUNT = TOURNAMENT_SIZE = POPULATION_SIZE // 4 (config.py:49-50)
        self.H = int(hof_size) if hof_size is not None else max(self.P // 4, 1)
        self.tournsize = int(tournsize) if tournsize is not None else max(self.P // 4, 1)
        if self.P < 1 or self.H < 0 or self.tournsize < 1:
            raise ValueError("population_size >= 1, hof_size >= 0 and tournsize >= 1 required")
        self.ev = D.Evaluator(self.nodes, bias=bias, dtype=dtype, device=device, n_games=n_games,
                              precision=precision, kernel=kernel, seed=physics_seed,
                              timeout_thresh=timeout_thresh, win_score=win_score)
        self.device, self.dtype, self.G = self.ev.device, dtype, self.ev.genes
        self.bias, self.n_games, self.schedule = bool(bias), int(n_games), schedule
        self.cxpb, self.mutpb, self.alpha = float(cxpb), float(mutpb), float(alpha)
        self.mu, self.sigma, self.indpb = float(mu), float(sigma), float(indpb)
        self.seed, self.physics_seed = int(seed), int(physics_seed)
        self.precision, self.kernel = precision, kernel
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.lo, self.hi = PD.shard_range(self.P, self.rank, self.world)
        # Self-play against a sliced hall (pg_schedule_args.hof_slices):
        # with hof_block_rows B > 0 the genomes of row block r // B play the hall's
        # interleaved slice (r // B) mod K, K = ceil(P / B) -- a function of the
        # global row, so any sharding plays the same games; a rank whose shard is
        # one block passes only its slice (1/K of the hall's lane records).  P <= B:
        # K = 1, the plain schedule.
        self.hof_block_rows = int(hof_block_rows)
        self.hof_slices = 1
        if self.hof_block_rows > 0 and schedule == "selfplay":
            self.hof_slices = max(1, min(-(-self.P // self.hof_block_rows), max(self.H, 1)))
        B = self.hof_block_rows
        # the slice k_schedule gives this block: (row // B) mod K (round-5 review:
        # without the mod a block index >= K named a slice the schedule never plays)
        self._slice = ((self.lo // B) % self.hof_slices
                       if self.hof_slices > 1 and self.hi > self.lo and self.lo // B == (self.hi - 1) // B else None)
        self.store = torch.zeros((self.H + self.P, self.G), dtype=dtype, device=self.device)
        self.spare = torch.empty_like(self.store)
        # the hall in place (fused path): the first buffer's hall rows, fixed
        # across the store/spare swaps; member j's row is _hall_buf[hof_slot[j]]
        self.in_place_hall = True
        self._hall_buf = self.store[: self.H]
        # the scan's upload lands here (fitness bits, sources, slots); its last
        # quarter is hof_slot itself, so the new slots need no copy of their own
        M = max(self.H, 1)
        self._up_dev = torch.zeros(4 * M, dtype=torch.int32, device=self.device)
        self.hof_slot = self._up_dev[3 * M:]
        self.hof_slot.copy_(torch.arange(M, dtype=torch.int32, device=self.device))
        self._hof_slot_h = np.zeros(0, np.int32)
        self._slots_identity = True
        self._up_keep = None
        self.fitness = torch.zeros(self.P, dtype=torch.float64, device=self.device)
        self.valid = torch.zeros(self.P, dtype=torch.bool, device=self.device)
        self.hof_fitness = torch.zeros(max(self.H, 1), dtype=torch.float64, device=self.device)
        self.hof_n = 0
        self._hof_fit_host = np.zeros(0, np.float64)   # HallOfFame.items order (best first)
        self.hof_hash = torch.zeros(max(self.H, 1), dtype=torch.int64, device=self.device)  # pg_row_hash
        self.generation = -1  # -1: the initial population is not evaluated yet
        self.logbook = []
        self.last = None       # EvalResult of the latest evaluation (this rank's rows)
        self.last_rows = None  # their population rows (int32, invalid first), None: the shard rows[lo:hi]
        self.last_count = None  # device int32 [1]: how many of last_rows were played (None: all)
        self.eval_events = None  # optional (start, end) HIP events recorded around the evaluation launch
        self.profile = None      # dict: when set, step() adds per-phase wall ms (with device syncs)
        self._t_mark = self._t_sub = 0.0
        self._next = None        # (generation, inv, inherited): offspring already varied into spare[H:]
        self.early_prep = True   # _early_prep: schedule + genome records during the hall-of-fame scan
        self.hard_log = None     # optional [cap, 8] int32: the evaluation's hard decisions (pg_eval_args.hard_log)
        # optional callable(g, rows, opponents, result), right after each evaluation; in the fused
        # path ``rows`` is the whole row buffer, of which (sharded) only this rank's shard
        # [lo, hi) and the rows result played (result indices -> last_rows) are current
        self.on_evaluate = None
        # Evaluation order: a genome's longest game sets when its last game ends,
        # and a long game started late sets the launch's tail.  Each row carries
        # the longest game of its lineage's last evaluation (a child inherits its
        # parent's); the shard's invalid rows are played longest-first.  Order
        # only: every game's result is the same in any order.
        self.order_by_length = True
        self.lineage_frames = torch.zeros(self.P, dtype=torch.float32, device=self.device)
        # the hall-of-fame update's device half by pg_hof_prepare (one native call:
        # candidates, hashes, ranks, classes); False: the same scan input from
        # torch ops (nonzero, stable sort, unique), kept as the cross-check
        self.native_prepare = True
        # the generation's device work around the evaluation in few native
        # launches and two host syncs (csrc/pg_gen.hip): False runs the torch
        # formulation above (the cross-check of tests/test_gpu_generation.py)
        self.fused = True
        # the fused path runs the next generation's select/vary beside the
        # hall-of-fame update on a second HIP stream (False: one stream, the A/B)
        self.side_stream = True
        self._side = None
        # the hall-of-fame prepare enqueued before the side stream's work (the
        # host's dispatch of that work then overlaps the device's prepare)
        self.prepare_first = True
        # unsharded: the next generation's side-stream work enqueued behind the
        # merge, before the host waits on it (_step_fused)
        self.presubmit = True
        self._pinned = {}  # name -> persistent pinned host buffer (_pin)
        # the schedule, invalid flags and remapped opponents in persistent
        # buffers (False: fresh tensors each generation, the A/B)
        self.persistent_bufs = True
        self._up_flip = 0
        self._iota_P = None  # (sharded presubmit: row positions, to bound the candidate list on the device)
        # sharded variation (module docstring; fused path): at N = 1 the shard is
        # the whole population and there is nothing to leave out
        self.shard_vary = self.world > 1
        # Length-balanced shards (fused path, N > 1; BASELINE config 5's strong
        # scaling): a generation's invalid rows, ordered longest predicted game
        # first over the whole population (the lineage is replicated: the
        # all-gather carries it), are dealt to the ranks in snake order, so every
        # rank plays an equal share of long and short genomes and the slowest
        # rank -- the generation's pace -- waits for no unlucky contiguous shard.
        # A rank still varies its contiguous shard (shard_rows() and
        # population_full() stay as they are) and also the rows dealt to it.
        self.balance_shards = False
        self._dealt = {}  # generation parity -> pair mask of the rows dealt to this rank
        self._n_pairs = (self.P + 1) // 2
        self._skip = (self.lo >> 1, (self.hi + 1) >> 1) if self.hi > self.lo else (0, 0)
        self._shard_pairs = None
        self.ws = D.Workspaces(self.device)
        self._lineage_alt = torch.zeros_like(self.lineage_frames)
        self._hof_hash_alt = torch.zeros_like(self.hof_hash)
        self._hof_fitness_alt = torch.zeros_like(self.hof_fitness)
        self._fit_alt = torch.zeros_like(self.fitness)
        self._summary_h = torch.zeros(8, dtype=torch.float64, pin_memory=True)

    # ------------------------------------------------------------ schedule
    def _sliced(self, n_hof: int) -> bool:
        return self._slice is not None and n_hof >= self.hof_slices

    def _opponents(self, buf: torch.Tensor, n_hof: int) -> Optional[torch.Tensor]:
        """The hall rows this rank's games index: the whole hall, or its slice
        (in place: the slots [0, n_hof) -- the schedule's positions go through
        _opp_slots -- or the slice's rows gathered in position order)."""
        if not n_hof:
            return None
        if self._in_place():
            if self._sliced(n_hof):
                idx = self.hof_slot[self._slice:n_hof:self.hof_slices].long()
                out = self._buf("hall_slice", (idx.shape[0], self.G), self.dtype)
                torch.index_select(self._hall_buf, 0, idx, out=out)
                return out
            return self._hall_buf[:n_hof]
        return buf[self._slice:n_hof:self.hof_slices] if self._sliced(n_hof) else buf[:n_hof]

    def _in_place(self) -> bool:
        return bool(self.in_place_hall and self.fused and self.H > 0)

    def _opp_slots(self, opp: torch.Tensor, n_hof: int) -> torch.Tensor:
        """The schedule's hall positions as the in-place hall's slots (a sliced
        hall's local indices need nothing: its rows were gathered in order)."""
        if not self._in_place() or not n_hof or self._sliced(n_hof) or self._slots_identity:
            return opp
        out = self._buf("opp_slots", opp.numel(), torch.int32) if self.persistent_bufs else None
        return torch.index_select(self.hof_slot[:n_hof], 0, opp.reshape(-1), out=out).view_as(opp)

    def _opponents_by_position(self, n_hof: int) -> Optional[torch.Tensor]:
        """The opponents in the schedule's index order (for on_evaluate)."""
        if not n_hof:
            return None
        if self._in_place() and not self._sliced(n_hof):
            return self.hall_of_fame[:n_hof]
        return self._opponents(self.store, n_hof)

    def eval_schedule(self, g: int, n_hof: Optional[int] = None, rows="last", out: Optional[tuple] = None):
        """(kind, opp, mult) of generation g's games for this rank's shard,
        as the evaluation plays them (opp indexes the opponents the evaluation
        passes -- the hall, or this rank's slice of it; rows: the evaluation
        order, by default the last evaluation's; out: the tensors to write)."""
        n_hof = self.hof_n if n_hof is None else n_hof
        rows = self.last_rows if isinstance(rows, str) else rows
        kw = {}
        if self.hof_slices > 1:
            kw = dict(hof_slices=self.hof_slices, block_rows=self.hof_block_rows, slice_local=self._sliced(n_hof))
        n = rows.shape[0] if rows is not None else self.hi - self.lo
        return D.schedule(self.schedule, n, self.n_games, self.lo, self.hof_fitness, n_hof, self.seed,
                          g, self.device, rows=rows, out=out, **kw)

    def _sched_bufs(self, g: int, n: int) -> tuple:
        """Generation g's schedule tensors, by generation parity (the next
        generation's schedule is made while this one's evaluation may still
        read it); persistent, so no side-stream allocation is freed across streams."""
        if not self.persistent_bufs:
            return None
        return (self._buf("sched_kind%d" % (g & 1), (n, self.n_games), torch.int32),
                self._buf("sched_opp%d" % (g & 1), (n, self.n_games), torch.int32),
                self._buf("sched_mult%d" % (g & 1), (n, self.n_games), torch.float64))

    def _balanced(self) -> bool:
        # (not with a sliced hall: there a rank's opponents are its row block's slice)
        return bool(self.balance_shards and self.fused and self.world > 1 and dist.is_initialized()
                    and self.hof_slices == 1)

    @property
    def _n_eval(self) -> int:
        """Entries of this rank's evaluation: its shard, or (balanced) ceil(P / N) dealt rows."""
        return -(-self.P // self.world) if self._balanced() else self.hi - self.lo

    # ------------------------------------------------------------ views
    @property
    def _rows(self) -> torch.Tensor:
        """Every population row of the device buffer (internal: with sharded
        variation only this rank's shard, the hall-of-fame candidates and the
        next parents are current)."""
        return self.store[self.H:]

    @property
    def population(self) -> torch.Tensor:
        """The current population [P, G] (the reference's ``ga.population``).
        With sharded variation (N > 1, ``shard_vary``) a rank holds only its
        shard's rows current, so this raises instead of returning stale rows:
        use :meth:`shard_rows` (this rank's rows, no communication) or
        :meth:`population_full` (a collective)."""
        if self._sharded():
            raise RuntimeError("DeviceGA.population: with sharded variation this rank holds only its shard "
                               "current; use shard_rows() or population_full() (a collective)")
        return self._rows

    def shard_rows(self) -> torch.Tensor:
        """This rank's shard of the population, rows [lo, hi) (always current)."""
        return self._rows[self.lo:self.hi]

    def population_full(self) -> torch.Tensor:
        """The whole current population on this rank: ``population`` itself, or
        with sharded variation the ranks' shard rows all-gathered (a
        collective: every rank calls it)."""
        if not self._sharded():
            return self._rows
        return PD.gather_rows(self._rows[self.lo:self.hi].contiguous(), self.P, self.group)

    def population_hash(self) -> torch.Tensor:
        """pg_row_hash of every population row ([P] int64; sharded: each rank
        hashes its shard and the 8-B hashes are all-gathered)."""
        if not self._sharded():
            return D.row_hash(self._rows, self.G)
        return PD.gather_rows(D.row_hash(self._rows[self.lo:self.hi], self.G), self.P, self.group)

    def _sharded(self) -> bool:
        return bool(self.shard_vary and self.fused and self.world > 1 and dist.is_initialized())

    @property
    def hall_of_fame(self) -> torch.Tensor:
        """Members, best first (HallOfFame.items order); the in-place hall's
        rows gathered in that order (a copy)."""
        if self._in_place():
            return self._hall_buf[self.hof_slot[: self.hof_n].long()]
        return self.store[: self.hof_n]

    @property
    def hof_member_fitness(self) -> np.ndarray:
        return self._hof_fit_host.copy()

    # ------------------------------------------------------------ state
    def initialize(self, init: str = "uniform", init_sigma: float = 3.0):
        """toolbox.population(n=P): genes U[0,1) as toolbox.attr_float = random.random
        (ga.py:85), or N(0, init_sigma) ("normal"), drawn on device in row blocks."""
        gen = torch.Generator(device=self.device).manual_seed(self.seed)
        rows = max(1, (1 << 28) // (8 * self.G))
        for r0 in range(0, self.P, rows):
            r1 = min(self.P, r0 + rows)
            if init == "uniform":
                blk = torch.rand((r1 - r0, self.G), generator=gen, dtype=torch.float64, device=self.device)
            elif init == "normal":
                blk = torch.randn((r1 - r0, self.G), generator=gen, dtype=torch.float64,
                                  device=self.device).mul_(init_sigma)
            else:
                raise ValueError("init must be 'uniform' or 'normal'")
            self.store[self.H + r0:self.H + r1] = blk.to(self.dtype)
        self.valid.zero_()
        self.fitness.zero_()
        self._set_hof_empty()
        self._next = None
        self.generation = -1
        self.logbook = []

    def set_population(self, genomes: torch.Tensor, fitness: Optional[torch.Tensor] = None,
                       valid: Optional[torch.Tensor] = None):
        """Load P genomes (and, for individuals whose fitness is valid, their fitness)."""
        if tuple(genomes.shape) != (self.P, self.G):
            raise ValueError(f"genomes must be [{self.P}, {self.G}], got {tuple(genomes.shape)}")
        self._next = None
        self._rows.copy_(genomes.to(device=self.device, dtype=self.dtype))
        if fitness is None:
            self.valid.zero_()
            self.fitness.zero_()
        else:
            self.fitness.copy_(fitness.to(device=self.device, dtype=torch.float64))
            v = torch.ones(self.P, dtype=torch.bool) if valid is None else valid.to(torch.bool)
            self.valid.copy_(v.to(self.device))

    def set_hall_of_fame(self, genomes: Optional[torch.Tensor], fitness):
        """Load hall-of-fame members, best first (HallOfFame.items order);
        ``genomes`` None: the members were written into hall-of-fame rows
        ``store[:n]`` in place."""
        fit = np.asarray(fitness, dtype=np.float64)
        n = fit.shape[0]
        if n > self.H or (genomes is not None and tuple(genomes.shape) != (n, self.G)):
            raise ValueError(f"hall of fame must be [<= {self.H}, {self.G}] with matching fitness")
        if n and np.any(np.diff(fit) > 0):
            raise ValueError("hall-of-fame members must be ordered best first")
        if genomes is not None:
            self.store[:n] = genomes.to(device=self.device, dtype=self.dtype)
        # a prepared next generation (_early_prep) assumed the old hall's size
        self._next = None
        self.hof_n = n
        self._hof_fit_host = fit.copy()
        # the in-place hall: slots = positions again, its rows from store[:n]
        if n and self._hall_buf.data_ptr() != self.store.data_ptr():
            self._hall_buf[:n] = self.store[:n]
        if self.H:
            self.hof_slot.copy_(torch.arange(self.hof_slot.shape[0], dtype=torch.int32, device=self.device))
        self._hof_slot_h = np.arange(n, dtype=np.int32)
        self._slots_identity = True
        if n:
            self.hof_fitness[:n] = torch.from_numpy(fit).to(self.device)
            self.hof_hash[:n] = D.row_hash(self.store[:n], self.G)

    def _set_hof_empty(self):
        self.hof_n = 0
        self._hof_fit_host = np.zeros(0, np.float64)
        self._hof_slot_h = np.zeros(0, np.int32)
        self._slots_identity = True

    # ------------------------------------------------------------ steps
    def _evaluate(self, g: int, rows: torch.Tensor, inv: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Fitness of the rows of ``rows`` ([P, G]) that eaSimple evaluates:
        those ``inv`` marks (``invalid_ind``, main.py:165-170; every row if
        None; the others' entries are 0).  Rank r plays the invalid rows of its
        shard ``shard_range(P, r, N)`` and the shards' fitness is all-gathered
        -- the generation's one collective.  The shard's invalid rows are
        compacted on the device and the launch reads their count from device
        memory (pg_eval_args.n_active), so no host round trip precedes it."""
        lo, hi = self.lo, self.hi
        n = hi - lo
        local = count = None
        if inv is not None:
            inv_s = inv[lo:hi]
            c_inv = torch.cumsum(inv_s, 0, dtype=torch.int32)
            count = c_inv[-1:] if n else torch.zeros(1, dtype=torch.int32, device=self.device)
            if self.order_by_length:
                # invalid rows first, longest predicted game first (clones key -1, last)
                key = torch.where(inv_s, self.lineage_frames[lo:hi], torch.full_like(self.lineage_frames[lo:hi], -1.0))
                local = (torch.argsort(key, descending=True, stable=True) + lo).to(torch.int32)
            else:
                c_val = torch.cumsum(~inv_s, 0, dtype=torch.int32)
                dest = torch.where(inv_s, c_inv - 1, count + c_val - 1).long()
                local = torch.empty(n, dtype=torch.int32, device=self.device)
                local[dest] = torch.arange(lo, hi, dtype=torch.int32, device=self.device)  # invalid rows first
        kind, opp, mult = self.eval_schedule(g, rows=local)
        opponents = self._opponents(self.store, self.hof_n)
        out = self.last if (self.last is not None and self.last.fitness.shape[0] == n) else None
        if self.eval_events is not None:
            self.eval_events[0].record()
        if local is None:
            res, _ = self.ev.evaluate(rows[lo:hi], kind, opp, mult, opponents=opponents, out=out, validate=False,
                                      hard_log=self.hard_log)
        else:
            res, _ = self.ev.evaluate(rows, kind, opp, mult, opponents=opponents, out=out, validate=False,
                                      hard_log=self.hard_log, rows=local, n_active=count)
        if self.eval_events is not None:
            self.eval_events[1].record()
        self.last, self.last_rows, self.last_count = res, local, count
        if self.on_evaluate is not None:
            self.on_evaluate(g, rows if local is not None else rows[lo:hi], opponents, res)
        longest = res.frames.max(dim=1).values.to(torch.float32)
        if local is None:
            self.lineage_frames[lo:hi] = longest
        else:  # the played rows' longest games; clones keep their lineage's
            played = torch.arange(n, device=self.device) < count
            at = local.long()
            self.lineage_frames[at] = torch.where(played, longest, self.lineage_frames[at])
        fit = res.fitness
        if local is not None:  # back to shard order; rows not played (clones) read 0
            shard = torch.zeros(n, dtype=torch.float64, device=self.device)
            shard[local.long() - lo] = fit
            fit = torch.where(inv_s, shard, torch.zeros_like(shard))
        # with a process group the all-gather runs at any world size (at N = 1 a
        # one-rank RCCL collective: the N > 1 code path, exercised on one GPU)
        return PD.gather_fitness(fit, self.P, self.group) if dist.is_initialized() else fit

    @staticmethod
    def _check(fit: torch.Tensor):
        # a NaN fitness is a game whose calculate_reward divided by zero (utils.py:106-108)
        if bool(torch.isnan(fit).any()):
            raise ZeroDivisionError("float division by zero (calculate_reward with total_frames == 0)")

    def _select_vary(self, g: int, parents: torch.Tensor, fitness: torch.Tensor, out: torch.Tensor):
        """Generation g's selTournament + varAnd into ``out``: returns (inv, inherited)."""
        chosen = D.select_tournament_ranked(fitness, self.P, self.tournsize, seed=self.seed, generation=g)
        _, invalid = D.vary(parents, chosen, self.G, self.cxpb, self.mutpb, self.alpha, self.mu,
                            self.sigma, self.indpb, seed=self.seed, generation=g, out=out)
        inherited = fitness[chosen.long()]  # a clone keeps its parent's fitness (varAnd)
        self.lineage_frames = self.lineage_frames[chosen.long()]  # and its parent's game lengths
        return invalid.bool(), inherited

    def _hof_update(self, fit: torch.Tensor, rows: torch.Tensor, dst: torch.Tensor, overlap=None):
        """HallOfFame.update(rows) with fitness ``fit``; the members are gathered
        into dst[:new_n] (dst is disjoint from the current members and rows).
        ``overlap`` (a callable enqueueing device work that touches none of
        these rows) runs once the host scan's inputs are copied out, so the
        device executes it while the host scans."""
        if self.H == 0:
            if overlap:
                overlap()
            return
        old_n = self.hof_n
        # a full hall only admits fitness > its worst, and the worst only rises:
        # rows at or below today's worst can never enter
        worst = float(self._hof_fit_host[-1]) if old_n >= self.H else None
        if self.native_prepare:  # pg_hof_prepare: candidates, hashes, ranks, classes in one call
            k, cand, hashes, packed_d = D.hof_prepare(fit, worst, rows, self.G, self.hof_fitness[:old_n],
                                                      self.hof_hash[:old_n])
        elif worst is not None:
            cand = torch.nonzero(fit > worst).flatten()
        else:
            cand = torch.arange(self.P, device=self.device)
        if not self.native_prepare:
            k = int(cand.numel())
        if k == 0:
            dst[:old_n] = self.store[:old_n]
            if overlap:
                overlap()
            return
        # Everything the sequential scan needs, computed on the device and sent
        # in one copy: each entry's rank in ascending (fitness, age) order (in
        # age order the old members come oldest first, then the candidates), a
        # dense similarity class per entry, and the candidates' fitness.
        n = old_n + k
        if self.profile is not None:
            self.profile["hof_candidates"] = self.profile.get("hof_candidates", 0) + k
        if not self.native_prepare:
            h = D.row_hash(rows, self.G, index=cand.to(torch.int32))
            fc = fit[cand]
            hashes = torch.cat([self.hof_hash[:old_n], h])
            by_age = torch.cat([self.hof_fitness[:old_n].flip(0), fc])
            order = torch.sort(by_age, stable=True).indices
            rank_age = torch.empty_like(order)
            rank_age[order] = torch.arange(n, device=self.device)
            rank = torch.cat([rank_age[:old_n].flip(0), rank_age[old_n:]])
            cls = torch.unique(hashes, return_inverse=True)[1]
            packed_d = torch.cat([rank | (cls << 32), fc.view(torch.int64)])
        packed_h = torch.empty(packed_d.shape, dtype=torch.int64, pin_memory=True)
        packed_h.copy_(packed_d, non_blocking=True)
        copied = torch.cuda.Event()
        copied.record()
        if overlap:
            overlap()
        copied.synchronize()
        packed = packed_h.numpy()
        self._mark("hof_prepare", sub=True)
        rank_np = (packed[:n] & 0xFFFFFFFF).astype(np.int32)
        cls_np = packed[:n] >> 32
        src, new_fit = D.hof_update(self.H, self._hof_fit_host, cls_np[:old_n], packed[n:].view(np.float64),
                                    cls_np[old_n:], rank=rank_np)
        self._mark("hof_scan", sub=True)
        m = src.shape[0]
        # one pinned upload: the members' fitness bits, then their sources
        up = torch.empty(3 * m, dtype=torch.int32, pin_memory=True)
        upn = up.numpy()
        upn[: 2 * m].view(np.float64)[:] = new_fit
        upn[2 * m:] = src
        up_d = up.to(self.device, non_blocking=True)
        src_t = up_d[2 * m:]
        D.gather_rows(dst, self.store, rows, src_t, old_n, index=cand)
        self.hof_hash[:m] = hashes.index_select(0, src_t.long())
        self.hof_fitness[:m] = up_d[: 2 * m].view(torch.float64)
        self.hof_n = int(m)
        self._hof_fit_host = new_fit

    @staticmethod
    def _summary(fit: torch.Tensor, invalid: torch.Tensor):
        """One device->host sync for the generation's host-side needs: whether
        any fitness is NaN, the logbook statistics and nevals."""
        v = torch.stack([torch.isnan(fit).any().double(), fit.mean(), fit.std(unbiased=False), fit.min(), fit.max(),
                         invalid.sum().double()]).tolist()
        if v[0]:
            # a NaN fitness is a game whose calculate_reward divided by zero (utils.py:106-108)
            raise ZeroDivisionError("float division by zero (calculate_reward with total_frames == 0)")
        return v[1:5], int(v[5])

    def _record(self, g: int, nevals: int, vals=None) -> dict:
        if vals is None:
            f = self.fitness
            vals = torch.stack([f.mean(), f.std(unbiased=False), f.min(), f.max()]).tolist()
        rec = {"gen": g, "nevals": nevals, **dict(zip(STAT_FIELDS, vals))}
        self.logbook.append(rec)
        return rec

    def step(self) -> dict:
        """One eaSimple generation (or, first, the initial evaluation); returns the logbook row."""
        return self._step_fused() if self.fused else self._step_torch()

    def _step_torch(self) -> dict:
        if self.generation < 0:
            fit = self._evaluate(0, self._rows, ~self.valid)
            nevals = int((~self.valid).sum())
            new_fit = torch.where(self.valid, self.fitness, fit)
            self._check(new_fit)
            self.fitness, self.valid = new_fit, torch.ones_like(self.valid)
            # generation 1's offspring go to spare[H:] (no swap after the initial update)
            self._hof_update(new_fit, self._rows, self.spare,
                             overlap=lambda: self._prefetch(1, self._rows, new_fit, self.spare))
            self.store[: self.hof_n] = self.spare[: self.hof_n]
            self.generation = 0
            return self._record(0, nevals)
        g = self.generation + 1
        self._mark(None)
        off = self.spare[self.H:]
        if self._next is not None and self._next[0] == g:
            inv, inherited = self._next[1:]  # selected and varied during the previous hall-of-fame scan
        else:
            inv, inherited = self._select_vary(g, self._rows, self.fitness, off)
        self._next = None
        self._mark("select_vary")
        fit = self._evaluate(g, off, inv)  # invalid_ind only: clones keep their parent's fitness
        new_fit = torch.where(inv, fit, inherited)
        self._mark("evaluate")
        stats, nevals = self._summary(new_fit, inv)
        # generation g + 1's parents are this offspring; its offspring go to
        # store[H:] (this generation's parents, free now), the buffer the swap
        # below makes next step's spare[H:]
        self._hof_update(new_fit, off, self.spare, overlap=lambda: self._prefetch(g + 1, off, new_fit, self.store))
        self._mark("hall_of_fame")
        self.fitness = new_fit
        self.store, self.spare = self.spare, self.store
        self.generation = g
        rec = self._record(g, nevals, stats)
        self._mark("record")
        return rec

    # ------------------------------------------------- fused generation path
    # One generation = [prefetched: select, vary, inherit, order] -> schedule +
    # evaluation -> scatter (+ all-gather) -> merge (new fitness, statistics,
    # candidates) -> sync 1 -> candidates' hashes, ranks, classes -> sync 2,
    # with the next generation's select/vary/inherit/order enqueued meanwhile
    # -> host scan -> one upload -> commit.  Same semantics as _step_torch
    # (population, fitness, hall of fame equal; the statistics' last bits may
    # differ: they are reduced in a fixed order of their own).
    def _buf(self, name, shape, dtype):
        return self.ws.tensor(name, shape, dtype)

    def _select(self, g: int, fitness: torch.Tensor) -> torch.Tensor:
        """Generation g's selTournament (rows of generation g - 1), in the
        buffer of g's parity: generation g - 1's stays readable meanwhile."""
        chosen = self._buf("chosen%d" % (g & 1), self.P, torch.int32)
        D.select_ranked(fitness, self.P, self.tournsize, self.seed, g, self.ws, chosen=chosen)
        return chosen

    def _shard_mask(self) -> torch.Tensor:
        """The pairs of this rank's shard rows (fixed for the run)."""
        if self._shard_pairs is None:
            self._shard_pairs = torch.zeros(self._n_pairs, dtype=torch.uint8, device=self.device)
            self._shard_pairs[self._skip[0]:self._skip[1]] = 1
        return self._shard_pairs

    def _complete(self, g: int, off: torch.Tensor, parents: torch.Tensor, rows: torch.Tensor, name: str,
                  exclude: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Sharded variation: generation g's rows ``rows`` of ``off`` beyond this
        rank's shard (and beyond the pairs ``exclude`` marks), varied from
        generation g - 1's rows ``parents`` (their parents: rows an earlier
        completion made current) with generation g's selection; returns the
        pair mask written."""
        mask = self._buf("complete_" + name, self._n_pairs, torch.uint8)
        mask.zero_()
        D.mark_pairs(mask, rows, skip=self._skip, exclude=exclude)
        # the marked pairs as a compact list: one wave per marked pair, not per pair
        lst = self._buf("complete_list_" + name, self._n_pairs, torch.int32)  # (per name: two streams)
        cnt = self._buf("complete_count_" + name, 1, torch.int32)
        D.list_pairs(mask, lst, cnt)
        chosen = self._buf("chosen%d" % (g & 1), self.P, torch.int32)
        D.vary(parents, chosen, self.G, self.cxpb, self.mutpb, self.alpha, self.mu, self.sigma, self.indpb,
               seed=self.seed, generation=g, out=off, pair_list=(lst, cnt, min(rows.numel(), self._n_pairs)),
               invalid=self._buf("complete_inv_" + name, self.P, torch.uint8))
        return mask

    def _deal(self, inv_u8: torch.Tensor, g: int):
        """Length-balanced shards: this rank's evaluation order (rows, count) --
        the invalid rows of the whole population longest lineage first (ties by
        row, pg_ga_order), dealt in snake order over the ranks (dist.deal_positions)."""
        P = self.P
        grows = self._buf("deal_rows", P, torch.int32)
        gcount = self._buf("deal_count", 1, torch.int32)
        D.order(P, 0, inv_u8, self.lineage_frames, True, grows, gcount, self.ws)
        n = self._n_eval
        pos = PD.deal_positions(n, self.rank, self.world, self.device)
        local = self._buf("local_rows%d" % (g & 1), n, torch.int32)
        local.copy_(grows[pos.clamp(max=P - 1)])
        count = self._buf("local_count%d" % (g & 1), 1, torch.int32)
        count.copy_((pos < gcount.long()).sum().to(torch.int32).reshape(1))  # a prefix: pos grows with k
        return local, count

    def _gather_dealt(self, res, local: torch.Tensor, count: torch.Tensor) -> torch.Tensor:
        """The balanced evaluation's all-gather: every rank's (row, fitness,
        longest game) entries, scattered into the population's fitness (rows
        nobody played read 0) and lineage (played rows' longest games)."""
        P, n = self.P, local.shape[0]
        played = torch.arange(n, device=self.device) < count
        rid = torch.where(played, local.long(), torch.full_like(local, P, dtype=torch.int64))
        longest = res.frames.max(dim=1).values.double()
        pack = torch.stack([rid.double(), res.fitness, longest], dim=1)
        allp = PD.gather_equal(pack, self.group)
        at = allp[:, 0].long()  # (unplayed entries land in the dropped slot P)
        fit = torch.zeros(P + 1, dtype=torch.float64, device=self.device)
        fit.index_copy_(0, at, allp[:, 1])
        lin = torch.cat([self.lineage_frames, self.lineage_frames.new_zeros(1)])
        lin.index_copy_(0, at, allp[:, 2].float())
        self.lineage_frames.copy_(lin[:P])
        return fit[:P]

    def _next_gen_prep(self, g: int, parents: torch.Tensor, fitness: torch.Tensor, store: torch.Tensor,
                       cand_pairs: Optional[torch.Tensor] = None):
        """Generation g's selTournament + varAnd into store[H:] (sharded: this
        rank's shard rows), what the clones inherit, and the shard's
        evaluation order; kept in self._next.  Sharded, after generation
        g - 1's evaluation (``cand_pairs``: the pairs its candidates' completion
        wrote): first generation g - 1's rows that this selection picked as
        parents, from store[H:] (generation g - 2) before it is overwritten."""
        chosen = self._select(g, fitness)
        if cand_pairs is not None:
            # generation g - 1's pairs already current here: the shard's (skip), the
            # candidates' and (balanced) the rows dealt to this rank
            prev = self._dealt.get((g - 1) & 1)
            self._complete(g - 1, parents, store[self.H:], chosen, "parents",
                           exclude=cand_pairs if prev is None else (cand_pairs | prev))
        _, inv = D.vary(parents, chosen, self.G, self.cxpb, self.mutpb, self.alpha, self.mu, self.sigma, self.indpb,
                        seed=self.seed, generation=g, out=store[self.H:],
                        pair_mask=self._shard_mask() if self._sharded() else None,
                        invalid=self._buf("invalid%d" % (g & 1), self.P, torch.uint8) if self.persistent_bufs else None)
        inherited = self._buf("inherited", self.P, torch.float64)
        D.inherit(chosen, fitness, inherited, self.lineage_frames, self._lineage_alt)
        self.lineage_frames, self._lineage_alt = self._lineage_alt, self.lineage_frames
        if self._balanced():
            order = self._deal(inv, g)
            if self._sharded():  # the dealt rows beyond the shard, varied like a completion
                self._dealt[g & 1] = self._complete(g, store[self.H:], parents, order[0], "dealt%d" % (g & 1))
        else:
            order = self._order(inv, g)
        self._next = (g, inv, inherited, order, self._early_prep(g, store[self.H:], order))

    def _early_prep(self, g: int, off: torch.Tensor, order):
        """Generation g's schedule and its genomes' lane records, made before the
        hall-of-fame scan (the device is idle during it) when neither needs the
        updated hall of fame: a self-play schedule against a full hall of fame
        (its size stays H, and self-play opponents are picked by index only).
        Returns the schedule for _evaluate_fused, or None."""
        n = self._n_eval
        if (not self.early_prep or self.schedule != "selfplay" or self.H == 0 or self.hof_n != self.H or self.last is None
                or self.last.fitness.shape[0] != n):
            return None
        local, count = order
        sched = self.eval_schedule(g, n_hof=self.H, rows=local, out=self._sched_bufs(g, n))
        # the records land in the evaluator's workspace; the later PG_PREP_REST call
        # (same genomes, rows, count; opponents of the same size) adds the opponents'
        # (the opponents' rows are not read by a "genomes" preparation: the
        # current hall stands in for the updated one, which has the same size)
        opponents = self._hall_buf[: self.H] if self._in_place() else self._opponents(self.spare, self.H)
        if self._in_place() and self._sliced(self.H):
            opponents = self._hall_buf[self._slice:self.H:self.hof_slices]
        self.ev.evaluate(off, *sched, opponents=opponents, out=self.last, validate=False,
                         hard_log=self.hard_log, rows=local, n_active=count, prep="genomes")
        return sched

    def _order(self, inv_u8: Optional[torch.Tensor], g: int = 0):
        # by generation parity: generation g + 1's order is made while
        # generation g's (self.last_rows / last_count) is still read
        n = self.hi - self.lo
        local = self._buf("local_rows%d" % (g & 1), n, torch.int32)
        count = self._buf("local_count%d" % (g & 1), 1, torch.int32)
        D.order(n, self.lo, inv_u8, self.lineage_frames, self.order_by_length, local, count, self.ws)
        return local, count

    def _evaluate_fused(self, g: int, rows: torch.Tensor, order, sched=None) -> torch.Tensor:
        lo, hi = self.lo, self.hi
        n = self._n_eval
        local, count = order
        if sched is None:
            kind, opp, mult = self.eval_schedule(g, rows=local, out=self._sched_bufs(g, n))
        else:  # made during the hall-of-fame scan with the genomes' records (_early_prep)
            kind, opp, mult = sched
        opponents = self._opponents(self.store, self.hof_n)
        opp = self._opp_slots(opp, self.hof_n)
        out = self.last if (self.last is not None and self.last.fitness.shape[0] == n) else None
        if self.eval_events is not None:
            self.eval_events[0].record()
        res, _ = self.ev.evaluate(rows, kind, opp, mult, opponents=opponents, out=out, validate=False,
                                  hard_log=self.hard_log, rows=local, n_active=count,
                                  prep="all" if sched is None else "rest")
        if self.eval_events is not None:
            self.eval_events[1].record()
        self.last, self.last_rows, self.last_count = res, local, count
        if self.on_evaluate is not None:
            self.on_evaluate(g, rows, self._opponents_by_position(self.hof_n), res)
        if self._balanced():
            return self._gather_dealt(res, local, count)
        shard = self._buf("shard_fit", n, torch.float64)
        D.scatter_fitness(res, n, lo, local, count, shard, self.lineage_frames)
        if not dist.is_initialized():
            return shard
        # the fitness all-gather also carries each row's longest game, so every
        # rank orders its next shard from the same predictions
        both = torch.stack([shard, self.lineage_frames[lo:hi].double()], dim=1)
        full = PD.gather_fitness(both, self.P, self.group)
        self.lineage_frames.copy_(full[:, 1].float())
        return full[:, 0].contiguous()

    def _merge(self, fit: torch.Tensor, inv: Optional[torch.Tensor], inherited: Optional[torch.Tensor],
               worst: Optional[float]):
        """pg_ga_merge_fitness + the generation's first sync: (new fitness,
        candidates, their fitness, stats, nevals, k)."""
        new_fit, cand, cand_fit, ev = self._merge_start(fit, inv, inherited, worst)
        return (new_fit, cand, cand_fit) + self._merge_finish(ev)

    def _merge_start(self, fit, inv, inherited, worst):
        """pg_ga_merge_fitness enqueued with its summary's copy: (new fitness,
        candidates, their fitness, the event after the copy)."""
        new_fit = self._fit_alt
        cand = self._buf("cand", self.P, torch.int32)
        cand_fit = self._buf("cand_fit", self.P, torch.float64)
        summ = self._buf("summary", 8, torch.float64)
        D.merge_fitness(fit, inv, inherited, new_fit, worst, cand, cand_fit, summ, self.ws)
        self._summary_h.copy_(summ, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return new_fit, cand, cand_fit, ev

    def _merge_finish(self, ev):
        """The generation's first sync: (stats, nevals, k) from the summary."""
        ev.synchronize()
        v = self._summary_h.tolist()
        if v[0]:
            # a NaN fitness is a game whose calculate_reward divided by zero (utils.py:106-108)
            raise ZeroDivisionError("float division by zero (calculate_reward with total_frames == 0)")
        self._fit_alt = self.fitness
        return v[1:5], int(v[5]), int(v[6])

    def _hof_update_fused(self, rows: torch.Tensor, cand: torch.Tensor, cand_fit: torch.Tensor, k: int,
                          dst: torch.Tensor, overlap=None):
        """HallOfFame.update over the k candidates (rows ``rows[cand]``); the
        members are written to dst[:new_n] (disjoint from the current members and rows)."""
        if self.H == 0:
            if overlap:
                overlap()
            return
        old_n = self.hof_n
        in_place = self._in_place()
        if k == 0:
            if not in_place:
                dst[:old_n] = self.store[:old_n]
            if overlap:
                overlap()
            return
        if self.profile is not None:
            self.profile["hof_candidates"] = self.profile.get("hof_candidates", 0) + k
        # the next generation's select/vary/inherit/order/early prep depend only
        # on this generation's fitness: on a side stream from here, beside the
        # candidates' prepare, the host scan and the commit (the buffers are
        # disjoint: they write store[H:], the update reads rows and store[:old_n]
        # and writes dst[:m]); the next evaluation waits for both streams.  The
        # prepare and its copy are enqueued first, so the device runs them while
        # the host enqueues the side stream's work
        main = torch.cuda.current_stream(self.device)
        side = ready = None
        if overlap and self.side_stream:
            if self._side is None:
                self._side = torch.cuda.Stream(self.device)
            side = self._side
            ready = torch.cuda.Event()
            ready.record(main)
            if not self.prepare_first:  # (the A/B: the side stream's work enqueued first)
                side.wait_event(ready)
                with torch.cuda.stream(side):
                    overlap()
                self._keep_on(main)
                overlap = None
        n = old_n + k
        cand, cand_fit = cand[:k], cand_fit[:k]
        cand_hash = self._buf("cand_hash", k, torch.int64)
        packed = self._buf("packed", n + k, torch.int64)
        D.hof_prepare_cand(self.hof_fitness[:old_n], self.hof_hash[:old_n], cand, cand_fit, rows, self.G, cand_hash,
                           packed, self.ws)
        packed_h = self._pin("packed", n + k, torch.int64)
        packed_h.copy_(packed, non_blocking=True)
        copied = torch.cuda.Event()
        copied.record()
        self._mark("hof_prepare", sub=True)  # (profiling only: these marks synchronise)
        if overlap and side is not None:
            side.wait_event(ready)
            with torch.cuda.stream(side):
                overlap()
            self._keep_on(main)
        elif overlap:
            overlap()
        if overlap:
            self._mark("next_select_vary", sub=True)
        copied.synchronize()
        # the scan straight on the device's packing, visiting only the hall's
        # tail and the candidates (pg_hof_update_packed, O(k log k)); its
        # outputs land in the pinned upload buffer: fitness, sources, slots.
        # Two such buffers alternate: this scan reads the last one's fitness
        # and slots, and an upload is done long before its buffer's next turn
        # (the generation in between waits on the device twice)
        M = max(self.H, 1)
        self._up_flip ^= 1
        up = self._pin("up%d" % self._up_flip, 4 * M, torch.int32)
        res = D.hof_update_packed(self.H, self._hof_fit_host, packed_h.numpy(), k, out=up.numpy(),
                                  slot_in=self._hof_slot_h if in_place else None, slots=in_place)
        src, new_fit = res[0], res[1]
        self._mark("hof_scan", sub=True)
        m = src.shape[0]
        up_d = self._up_dev
        up_d.copy_(up, non_blocking=True)  # (in place: the slots land in hof_slot)
        src_d, fit_d = up_d[2 * M:2 * M + m], up_d[: 2 * M].view(torch.float64)[:m]
        if in_place:
            slot_d = up_d[3 * M:3 * M + m]
            D.hof_commit(self._hall_buf, None, rows, cand, src_d, old_n, self.G, self.hof_hash, cand_hash,
                         self._hof_hash_alt, fit_d, self._hof_fitness_alt, dst_slot=slot_d)
            self._hof_slot_h = res[2]
            self._slots_identity = False
        else:
            D.hof_commit(dst, self.store, rows, cand, src_d, old_n, self.G, self.hof_hash, cand_hash,
                         self._hof_hash_alt, fit_d, self._hof_fitness_alt)
        self.hof_hash, self._hof_hash_alt = self._hof_hash_alt, self.hof_hash
        self.hof_fitness, self._hof_fitness_alt = self._hof_fitness_alt, self.hof_fitness
        self.hof_n = int(m)
        self._hof_fit_host = new_fit
        self._up_keep = up  # _hof_fit_host (and _hof_slot_h) are views of it
        if side is not None:
            main.wait_stream(side)

    def _pin(self, name: str, n: int, dtype) -> torch.Tensor:
        """A persistent pinned host buffer's first n entries (grown on demand)."""
        buf = self._pinned.get(name)
        if buf is None or buf.shape[0] < n or buf.dtype != dtype:
            buf = torch.empty(max(n, 1), dtype=dtype, pin_memory=True)
            self._pinned[name] = buf
        return buf[:n]

    def _keep_on(self, stream):
        """The side stream's fresh tensors in self._next are read on ``stream``
        later: tell the caching allocator (record_stream) so their memory is not
        handed out again before that work is done."""
        if self._next is None:
            return
        for t in self._next[1:]:
            for x in (t if isinstance(t, tuple) else (t,)):
                if isinstance(x, torch.Tensor) and x.is_cuda:
                    x.record_stream(stream)

    def _step_fused(self) -> dict:
        worst = float(self._hof_fit_host[-1]) if (self.H and self.hof_n >= self.H) else None
        if self.generation < 0:
            inv = (~self.valid).to(torch.uint8)
            fit = self._evaluate_fused(0, self._rows, self._deal(inv, 0) if self._balanced() else self._order(inv))
            new_fit, cand, cand_fit, stats, nevals, k = self._merge(fit, inv, self.fitness, worst)
            self.fitness, self.valid = new_fit, torch.ones_like(self.valid)
            # generation 1's offspring go to spare[H:] (no swap after the initial
            # update); the initial population is current on every rank
            self._hof_update_fused(self._rows, cand, cand_fit, k, self.spare,
                                   overlap=lambda: self._next_gen_prep(1, self._rows, new_fit, self.spare))
            if not self._in_place():
                self.store[: self.hof_n] = self.spare[: self.hof_n]
            self.generation = 0
            return self._record(0, nevals, stats)
        g = self.generation + 1
        self._mark(None)
        off = self.spare[self.H:]
        if self._next is None or self._next[0] != g:
            self._next_gen_prep(g, self._rows, self.fitness, self.spare)
        _, inv, inherited, order, sched = self._next
        self._next = None
        self._mark("select_vary")
        fit = self._evaluate_fused(g, off, order, sched)  # invalid_ind only: clones keep their parent's fitness
        new_fit, cand, cand_fit, merged = self._merge_start(fit, inv, inherited, worst)
        # The next generation's select/vary/inherit/order/early prep need only
        # this merge's fitness (and, sharded, the candidates' completion): they
        # are enqueued on the side stream now, behind the merge, while this
        # evaluation still runs -- the device starts them the moment the merge
        # ends, and the host's dispatch of them is off the path between two
        # evaluations.  Sharded, the candidates' completion goes first on the
        # main stream, over the candidate list bounded by the count the merge
        # left on the device (rows past it read -1, which marks no pair).
        early_side = self.side_stream and self.presubmit and not self._balanced()
        cand_pairs = None
        if early_side:
            main = torch.cuda.current_stream(self.device)
            if self._side is None:
                self._side = torch.cuda.Stream(self.device)
            after = merged
            if self._sharded():
                if self.H:
                    if self._iota_P is None:
                        self._iota_P = torch.arange(self.P, dtype=torch.float64, device=self.device)
                    k_dev = self._buf("summary", 8, torch.float64)[6]
                    rows_all = torch.where(self._iota_P < k_dev, cand, torch.full_like(cand, -1))
                else:
                    rows_all = cand[:0]  # (no hall of fame: the candidates are never read)
                cand_pairs = self._complete(g, off, self._rows, rows_all, "cand")
                after = torch.cuda.Event()
                after.record(main)
            self._side.wait_event(after)
            with torch.cuda.stream(self._side):
                self._next_gen_prep(g + 1, off, new_fit, self.store, cand_pairs)
            self._keep_on(main)
        stats, nevals, k = self._merge_finish(merged)
        self._mark("evaluate")
        if self._sharded() and not early_side:
            # the candidates' rows of this offspring beyond the shard (the update
            # hashes and gathers them); the next selection's parents follow on
            # the side stream (_next_gen_prep), both before generation g + 1's
            # variation overwrites store[H:]
            # (no hall of fame: the candidates are never read)
            cand_pairs = self._complete(g, off, self._rows, cand[:k] if self.H else cand[:0], "cand",
                                        exclude=self._dealt.get(g & 1) if self._balanced() else None)
            self._mark("complete", sub=True)
        # generation g + 1's parents are this offspring; its offspring go to
        # store[H:] (this generation's parents, free now), the buffer the swap
        # below makes next step's spare[H:]
        self._hof_update_fused(off, cand, cand_fit, k, self.spare,
                               overlap=None if early_side else
                               (lambda: self._next_gen_prep(g + 1, off, new_fit, self.store, cand_pairs)))
        if early_side:  # the next evaluation follows the side stream's work
            torch.cuda.current_stream(self.device).wait_stream(self._side)
        self._mark("hall_of_fame")
        self.fitness = new_fit
        self.store, self.spare = self.spare, self.store
        self.generation = g
        rec = self._record(g, nevals, stats)
        self._mark("record")
        return rec

    def _prefetch(self, g: int, parents: torch.Tensor, fitness: torch.Tensor, store: torch.Tensor):
        self._next = (g,) + self._select_vary(g, parents, fitness, store[self.H:])

    def _mark(self, phase, sub: bool = False):
        """Profiling: add the wall time since the last top-level mark to
        ``phase``; ``sub`` marks split a phase (since the last mark of either kind)."""
        if self.profile is None:
            return
        import time
        torch.cuda.synchronize(self.device)
        now = time.perf_counter()
        if sub:
            self.profile[phase] = self.profile.get(phase, 0.0) + (now - self._t_sub) * 1e3
            self._t_sub = now
            return
        if phase is not None:
            self.profile[phase] = self.profile.get(phase, 0.0) + (now - self._t_mark) * 1e3
        self._t_mark = self._t_sub = now

    def run(self, ngen: int, verbose: bool = False) -> list:
        """algorithms.eaSimple(..., ngen): the initial evaluation if pending, then ngen generations."""
        rows = []
        if self.generation < 0:
            rows.append(self.step())
            if verbose:
                _print_row(rows[-1], header=True)
        for _ in range(int(ngen)):
            rows.append(self.step())
            if verbose:
                _print_row(rows[-1], header=False)
        return rows


def _print_row(rec: dict, header: bool):
    cols = ("gen", "nevals") + STAT_FIELDS
    if header:
        print("\t".join(cols))
    print("\t".join(str(rec[c]) for c in cols))
