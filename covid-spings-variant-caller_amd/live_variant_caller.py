"""Drop-in ``LiveVariantCaller`` (variant_caller/live_variant_caller.py:21-297) on the MI355X engine.

Same constructor arguments, methods and semantics as the reference class:

* ``process_bam(inputBam, referenceIndex=0)`` (:54-72) — the contig's pileup is built by the host
  emulator (``pileup.AlignmentFile``, include/spings_pileup.h) with pysam's pileup() defaults and
  the caller's min_mapping_quality, then accumulated on the GPU (``spg_accumulate``) where the
  base-quality filter, ``process_pileup_column`` and ``process_svn`` (:74-103) run.  Accumulates
  across calls like ``memory``; positions are keyed by coordinate only, as in the reference.
* ``prepare_variants()`` (:120-231) — ``spg_finalize`` on the GPU; returns the reference's
  ``List[Variant]`` (start, stop, alleles, qual, info{DP, AD, GL, PL, SCORE}) in memory order.
* ``write_vcf(outputVfc)`` (:233-297) — same header, records sorted by (start, SCORE); written by
  pysam when it is importable, otherwise by a writer that emits the text htslib produces for this
  header (float32 QUAL/Float INFO printed with %g).
* ``reset_memory()`` (:37-38), ``create_checkpoint`` / ``load_checkpoint`` (:40-52) — the
  checkpoint holds the accumulated batches (the engine's exact state) instead of a pickle.
* ``memory`` (:32) — read-only view rebuilt from the device table and batch history.

Exceptions propagate like the reference's (missing files -> OSError, unknown contig ->
ValueError, engine/library failures -> RuntimeError).  There is no CPU path: without
libspings_gpu.so or a GPU the constructor raises.
"""
from __future__ import annotations

import collections
import uuid
import logging
import os
import threading
from collections.abc import Mapping
from typing import Dict, List, Optional

import numpy as np

from . import _native as N
from .engine import PileupEngine
from .pileup import AlignmentFile, PileupParams, cpu_share
from .structs import Site, Variant

log = logging.getLogger("covid_spings_variant_caller_amd")


class FastaFile:
    """The part of pysam.FastaFile the caller uses: references, lengths, fetch(reference=)."""

    def __init__(self, path: str):
        if not os.path.exists(path):
            raise FileNotFoundError(f"could not open fasta file `{path}`")
        self.filename = path
        self.references: List[str] = []
        self._seq: Dict[str, str] = {}
        name, parts = None, []
        with open(path) as f:
            for line in f:
                line = line.rstrip("\r\n")
                if line.startswith(">"):
                    if name is not None:
                        self._seq[name] = "".join(parts)
                    name, parts = line[1:].split()[0] if line[1:].split() else "", []
                    self.references.append(name)
                elif line:
                    parts.append(line.strip())
        if name is not None:
            self._seq[name] = "".join(parts)
        self.lengths = [len(self._seq[r]) for r in self.references]

    def fetch(self, reference: str) -> str:
        if reference not in self._seq:
            raise KeyError(f"sequence '{reference}' not present")
        return self._seq[reference]

    def get_reference_length(self, reference: str) -> int:
        return len(self.fetch(reference))

    def close(self):
        pass


class PinnedIngest:
    """Pinned host staging for process_bam (spg_host_alloc): two buffer sets used alternately, so the
    pileup of BAM k+1 is written into one set while BAM k's entries are still being copied to HBM from the
    other.  A set is reused only after ITS copy has landed (spg_wait_ticket on the ticket taken when it was
    enqueued); the copy of the other set, and kernels, keep running.  Pinned pages are DMA'd without a
    staging copy, take no page faults when reused, and let spg_accumulate return without a host sync."""

    def __init__(self, engine):
        self.engine = engine
        self.sets = [None, None]
        self.tickets = [0, 0]
        self.slot = 0

    def buffers(self, n_entries: int, n_cols: int):
        from .engine import pinned_empty
        s = self.slot
        need = int(n_entries) + 16
        cur = self.sets[s]
        self.engine.wait_ticket(self.tickets[s])   # this set's previous copy has landed
        if cur is None or cur[0].nbytes < need or cur[2].size < n_cols + 1:
            cap = max(need, int(need * 1.125))
            cur = (pinned_empty(cap), pinned_empty(cap), pinned_empty(int((n_cols + 1) * 1.125) + 1, np.uint64))
            self.sets[s] = cur
        return cur

    def enqueued(self):
        """The set returned by the last buffers() call has been handed to spg_accumulate."""
        self.tickets[self.slot] = self.engine.input_ticket()
        self.slot ^= 1


class MemoryView(Mapping):
    """``memory`` (live_variant_caller.py:32, dict[int, Site]) as a lazy mapping: iteration in insertion order (first
    visit) from the device table; a position's Site is built when it is read, from that position's entries over the
    history (spg_position_entries_upto: one device gather per lookup) — O(the position's entries), never O(all
    entries).  A snapshot: lookups see the batches accumulated when the view was taken, also after later process_bam
    calls (the view's totalDepth and quality lists stay consistent); a reset or a load invalidates it."""

    def __init__(self, order, depth, first_batch, refs, entries, min_bq, n_hist=None, valid=None):
        self._order = order
        self._sorted = np.sort(order)
        self._depth, self._fb, self._refs = depth, first_batch, refs
        self._entries, self._min_bq = entries, min_bq
        self._n_hist, self._valid = n_hist, valid

    def __len__(self):
        return len(self._order)

    def __iter__(self):
        return iter(self._order.tolist())

    def __contains__(self, p):
        i = np.searchsorted(self._sorted, p)
        return bool(i < len(self._sorted) and self._sorted[i] == p)

    def __getitem__(self, p) -> Site:
        if not isinstance(p, (int, np.integer)) or p not in self:
            raise KeyError(p)
        if self._valid is not None and not self._valid():
            raise RuntimeError("memory view taken before reset_memory / load_checkpoint: read memory again")
        p = int(p)
        codes, quals = self._entries(p, self._n_hist)
        keep = (quals >= self._min_bq) & (codes < 16)           # pileups' bq filter (:75, :89); D/N: depth only
        c, q = codes[keep], quals[keep]
        u, first = np.unique(c, return_index=True)
        snvs = {N.NIBBLE[int(k)]: q[c == k].tolist() for k in u[np.argsort(first)]}   # dict order = first seen
        return {"reference": self._refs[int(self._fb[p]) - 1][p], "totalDepth": int(self._depth[p]),
                "snvs": snvs, "indels": {}}


class LiveVariantCaller:
    def __init__(self, referenceFasta: str, minBaseQuality: int, minMappingQuality: int, minTotalDepth: int,
                 minAlleleDepth: int, minEvidenceRatio: float, maxVariants: int, device: Optional[int] = None,
                 max_depth: int = 8000, stepper: str = "all", ignore_overlaps: bool = True,
                 n_threads: Optional[int] = None, devices: Optional[List[int]] = None, pileup: str = "device",
                 gpu_inflate: bool = True, device_min_bytes: int = 32 << 20, checkpoint_write_behind: bool = False,
                 checkpoint_prealloc: bool = True, gpu_plan: bool = True):
        """The reference's 7 arguments (:22-32), then the engine's: ``device`` (default LOCAL_RANK or 0), or
        ``devices`` — several GPUs of this host, each owning a coordinate range of the contig (multi.MultiEngine,
        spg_multi_*: BAM records and host batches sliced at equal-entry cuts, one RCCL gather of the call tables);
        pileup()'s ``max_depth`` / stepper / ``ignore_overlaps``; host threads of the BAM plan.

        ``pileup`` — where a BAM's pileup is built (SAM input always takes "host"):
          "device"  (default) process_bam keeps the BAM in HBM: the compressed file goes up, the GPU inflates
                    and scans it, only the reads' fixed fields come down for the host's depth-cap / mate-pairing
                    replay, and the entries are written on the GPU (spg_bam_*); process_bams pipelines it over two
                    device BAM slots (the next BAM opens on the GPU while the host plans this one); multi-device
                    callers use the records plan below.  A BAM the device path cannot take (a member it cannot inflate,
                    record chains that disagree, a name-hash collision) falls back to the records plan, and so does
                    a BAM file smaller than ``device_min_bytes`` (default 32 MiB, ~1,300 BGZF members): the GPU
                    inflate takes ~19 ms however few members there are (one member's serial decode chain), which
                    the host's threads match at about that size (r05f: a 100x BAM took 20.6 ms on the device path,
                    ~2 ms on the records plan).
          "records" the host inflates and scans the BAM and takes the read decisions; the inflated records go to HBM
                    and the GPU decodes bases / qualities and walks the CIGARs (spg_accumulate_records);
          "host"    the host also writes every entry (spp_batch_fill) into pinned staging.
        ``gpu_inflate`` — records plans inflate BAMs of >= 4,096 BGZF members on this caller's (first) GPU
        (spg_bgzf_inflate) instead of on the host's threads.
        ``checkpoint_write_behind`` (default off: the reference's create_checkpoint returns with its file written) —
        create_checkpoint returns once the new batches are packed into pinned host memory; a helper thread writes the
        shard and then the manifest (a crash leaves the previous checkpoint, whole) while the caller moves on to the next
        BAM.  This caller's next create_checkpoint, reset_memory, close or flush_checkpoints(), and any caller's
        load_checkpoint of that file in this process, wait for it first (and raise the error it met, if any).
        ``checkpoint_prealloc`` (default on: vc_queue.py:134 checkpoints after every BAM) — a BAM kept in HBM reserves the
        pinned staging its checkpoint will need on a helper thread while the GPU works on it, so a caller's first
        create_checkpoint does not pin ~0.4 GB of pages itself.
        ``gpu_plan`` (default on) — a BAM kept in HBM has htslib's depth cap and mate pairing decided on the GPU
        (spg_bam_plan_build); off: its reads' fixed fields come down and the host replays them (spp_pileup_plan_fields),
        which is also the path of the rare BAMs the GPU plan declines."""
        if pileup not in ("device", "records", "host"):
            raise ValueError(f"pileup must be 'device', 'records' or 'host', not {pileup!r}")
        self.minBaseQuality = minBaseQuality
        self.minMappingQuality = minMappingQuality
        self.minTotalDepth = minTotalDepth
        self.minAlleleDepth = minAlleleDepth
        self.minEvidenceRatio = minEvidenceRatio
        self.maxVariants = maxVariants
        self.fastaFile = FastaFile(referenceFasta)
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        inflate_dev = (int(devices[0]) if devices else int(device)) if gpu_inflate else -1
        self.pileup_params = PileupParams(stepper=stepper, min_mapping_quality=minMappingQuality, max_depth=max_depth,
                                          ignore_overlaps=ignore_overlaps,
                                          n_threads=n_threads or min(16, cpu_share()), inflate_device=inflate_dev)
        n_pos = max(self.fastaFile.lengths) if self.fastaFile.lengths else 1
        # calls-only engine: prepare_variants() is the class's only statistical output
        if devices is not None and len(devices) > 0:
            from .multi import MultiEngine
            self.engine = MultiEngine(list(devices), max(len(devices), n_pos), minBaseQuality, minTotalDepth,
                                      minAlleleDepth, minEvidenceRatio, calls_only=True)
        else:
            self.engine = PileupEngine(max(1, n_pos), minBaseQuality, minTotalDepth, minAlleleDepth, minEvidenceRatio,
                                       device=device, calls_only=True)
        self._lock = threading.RLock()
        self._ingest = PinnedIngest(self.engine)
        self._batch_contig: List[int] = []       # FASTA reference index of each accumulated batch
        self.pileup = pileup
        self.device_pileup = pileup != "host"
        self._device_bam = pileup == "device" and devices is None
        self.device_min_bytes = int(device_min_bytes)
        self.last_bam_path = None                # which path the last BAM took: "device", "records" or "host"
        self.last_gpu_inflate = False
        if self.device_pileup:
            N.use_pinned_records()
        self._inflight = collections.deque()     # (input ticket, records plan) whose copy may still be running
        self._ck_bytes = 0                       # shard bytes the last create_checkpoint wrote
        self.checkpoint_write_behind = bool(checkpoint_write_behind)
        self.checkpoint_prealloc = bool(checkpoint_prealloc)
        self.gpu_plan = bool(gpu_plan)
        self.last_plan_path = None               # "device" (spg_bam_plan_build) or "host" (spp_pileup_plan_fields)
        self._ck_job = None                      # the write-behind checkpoint in flight (a Future)
        self._ck_pool = None
        self.reset_memory()

    def close(self):
        """Release the engine (HBM accumulators, history, BAM buffers) and this caller's GPU inflate scratch."""
        with self._lock:
            try:
                self.flush_checkpoints()
            finally:
                if self._ck_pool is not None:
                    self._ck_pool.shutdown(wait=True)
                    self._ck_pool = None
                self._drain()
                self.fastaFile.close()
                self.engine.close()
            if self.pileup_params.inflate_device >= 0:
                N.gpu_lib().spg_bgzf_release(self.pileup_params.inflate_device)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- memory -------------------------------------------------------------------------------
    def _drain(self, keep: int = 0):
        """Close the records plans whose inputs have landed in HBM (all but the newest ``keep``)."""
        while len(self._inflight) > keep:
            t, b = self._inflight.popleft()
            self.engine.wait_ticket(t)
            b.close()

    def reset_memory(self):
        """:37-38"""
        with self._lock:
            self.flush_checkpoints()
            self._drain()
            self.engine.reset()
            self._batch_contig = []
            self._current_ref = None
            self._ck_token = uuid.uuid4().hex     # identity of this memory for incremental checkpoints
            self._ck_chain = {}                   # directory -> this memory's shards there [(file, first, count)]

    def _use_reference(self, index: int):
        if self._current_ref != index:
            self.engine.set_reference(self.fastaFile.fetch(self.fastaFile.references[index]))
            self._current_ref = index

    @property
    def memory(self) -> Mapping[int, Site]:
        """Read-only view of the reference's ``memory`` (dict[int, Site], insertion order), as a lazy
        mapping: reference char and totalDepth from the device table, a position's per-allele quality lists
        (bq-filtered, BAM order, dict order of first appearance) gathered from the batch history on the device when
        the position is read (chr1 memories hold ~2.5e8 positions and ~7.5e9 entries)."""
        with self._lock:
            self.engine.finalize()
            t = self.engine.table()
            present = np.nonzero(t["flags"] & N.SPG_F_PRESENT)[0]
            order = present[np.lexsort((present, t["first_batch"][present]))]
            refs = [self.fastaFile.fetch(self.fastaFile.references[i]) for i in self._batch_contig]
            token = self._ck_token
            return MemoryView(order, t["depth"], t["first_batch"], refs, self.engine.position_entries,
                              self.minBaseQuality, n_hist=self.engine.history_count(),
                              valid=lambda: self._ck_token == token)

    # -- hot path -----------------------------------------------------------------------------
    def process_bam(self, inputBam: str, referenceIndex=0):
        """:54-72 — pileup of references[referenceIndex] accumulated on the GPU."""
        if not os.path.exists(inputBam):
            raise FileNotFoundError(f"[Errno 2] could not open alignment file `{inputBam}`: No such file or directory")
        contig = self.fastaFile.references[referenceIndex]
        with AlignmentFile(inputBam) as bam:
            if contig not in bam.references:
                raise ValueError(f"invalid contig `{contig}`")
            bgzf = _is_bgzf(inputBam)
            if (self._device_bam and bgzf and os.path.getsize(inputBam) >= self.device_min_bytes
                    and self._process_bam_device(bam, contig, referenceIndex, os.path.getsize(inputBam))):
                self.last_bam_path = "device"
                return
            if self.device_pileup and bgzf:
                batch = bam.pileup_records(contig, self.pileup_params)
                self.last_bam_path = "records"
            else:
                batch = bam.pileup_plan(contig, self.pileup_params)
                self.last_bam_path = "host"
        # the entries go straight into pinned staging (double-buffered): the copy to HBM runs on the engine's
        # copy stream while the next BAM is read
        self._accumulate_plan(batch, referenceIndex)

    def _process_bam_device(self, bam: AlignmentFile, contig: str, referenceIndex: int, file_bytes: int = 0) -> bool:
        """The BAM kept in HBM (spg_bam_*): compressed bytes up, inflate + record scan + stepper filter on the GPU, then
        htslib's depth cap / mate pairing decided on the GPU too (spg_bam_plan_build), mate-overlap tweak + entries +
        accumulate — nothing comes down.  When the device declines the plan (spg_bam_plan_build's rare cases), the kept
        reads' fixed fields come down and the host replays it (spp_pileup_plan_fields), the plan goes up.  False when
        the device declined the BAM itself (nothing accumulated: the caller plans it on the host)."""
        if self.checkpoint_prealloc and isinstance(self.engine, PileupEngine) and file_bytes:
            # the checkpoint's pinned staging for this BAM's batch, pinned on a helper thread while the GPU works (a
            # BAM's pileup entries are ~1.4 bytes per compressed byte here; vc_queue.py:134 checkpoints after every BAM)
            self.engine.reserve_staging(self.fastaFile.get_reference_length(contig) + 1, int(1.5 * file_bytes),
                                        write_behind=self.checkpoint_write_behind)
        bmap = bam.bam_map(self.pileup_params.n_threads)
        try:
            with self._lock:
                n = self.engine.bam_open(bmap, bam.tid(contig), self.pileup_params)
        finally:
            bmap.close()                         # (spg_bam_open has copied it)
        if n is None:
            log.info("device BAM path declined %s: %s", contig, self.engine.bam_fallback)
            return False
        with self._lock:
            if self.gpu_plan:
                plan = self.engine.bam_plan_build(self.pileup_params.max_depth, self.pileup_params.ignore_overlaps)
                if plan is not None:
                    self.last_plan_path = "device"
                    if plan.n_cols == 0:
                        return True
                    self._use_reference(referenceIndex)
                    if not self.engine.bam_accumulate_planned(plan):
                        log.info("device BAM plan declined: %s", self.engine.bam_fallback)
                        return False
                    self._batch_contig.append(referenceIndex)
                    return True
                log.info("GPU plan declined %s: %s (host plan)", contig, self.engine.bam_fallback)
            self.last_plan_path = "host"
            reads = self.engine.bam_reads(n)
            batch = bam.pileup_fields(contig, reads, self.pileup_params)
            if batch.n_cols == 0:
                batch.close()
                return True
            self._use_reference(referenceIndex)
            if not self.engine.bam_accumulate(batch):
                batch.close()
                log.info("device BAM plan declined: %s", self.engine.bam_fallback)
                return False
            # the plan's pinned arrays are copied on the engine's copy stream: keep them until that copy lands
            self._inflight.append((self.engine.input_ticket(), batch))
            self._drain(keep=2)
            self._batch_contig.append(referenceIndex)
        return True

    def process_bams(self, inputBams, referenceIndex=0, workers: Optional[int] = None):
        """vc_queue.py:142-144's loop of process_bam (:54-72) over many BAMs, as one call: the BAMs'
        pileups are planned on a thread pool (the C++ emulator, outside the GIL; each plan applies its own
        BAM's depth cap) a few BAMs ahead, and accumulated in the given order — first visits, dict order and
        history exactly as len(inputBams) process_bam calls.  A calls-only engine counts the whole run at the
        next prepare_variants (counted mode: k_acc_lite_run + the exact fold of the positions that can call)."""
        from concurrent.futures import ThreadPoolExecutor
        paths = list(inputBams)
        for f in paths:
            if not os.path.exists(f):
                raise FileNotFoundError(f"[Errno 2] could not open alignment file `{f}`: No such file or directory")
        import dataclasses
        contig = self.fastaFile.references[referenceIndex]
        if (self._device_bam and paths and
                all(_is_bgzf(f) and os.path.getsize(f) >= self.device_min_bytes for f in paths)):
            return self._process_bams_device(paths, contig, referenceIndex)
        # concurrent plans: one per 8 CPUs this process may use (the GPU box's 16-CPU quota: two), so one plan's serial
        # phases (record scan, depth-cap sweep) overlap the other's inflate; the host threads split between them
        workers = workers or max(1, min(4, cpu_share() // 8))
        params = dataclasses.replace(self.pileup_params, n_threads=max(1, self.pileup_params.n_threads // workers))

        def plan(path):
            with AlignmentFile(path) as bam:
                if contig not in bam.references:
                    raise ValueError(f"invalid contig `{contig}`")
                if self.device_pileup and _is_bgzf(path):
                    return bam.pileup_records(contig, params)
                return bam.pileup_plan(contig, params)

        window = workers + 1                  # plans in flight (each holds its BAM's inflated records, ~0.5 GB at 10,000x)
        self.last_gpu_inflate = self.device_pileup and self.pileup_params.inflate_device >= 0
        self.last_bam_path = "records" if self.device_pileup else "host"
        with ThreadPoolExecutor(workers) as ex:
            pending = [ex.submit(plan, p) for p in paths[:window]]
            for i in range(len(paths)):
                batch = pending[i].result()
                if i + window < len(paths):
                    pending.append(ex.submit(plan, paths[i + window]))
                pending[i] = None
                self._accumulate_plan(batch, referenceIndex)

    def _process_bams_device(self, paths, contig: str, referenceIndex: int):
        """process_bams with every BAM kept in HBM (as the lone process_bam), pipelined over the engine's two device BAM
        slots: BAM i + 1 is opened on the GPU (compressed bytes up, inflate, record scan, fields down) while the host
        replays BAM i's depth cap / mate pairing on a worker thread; BAM i is then accumulated, before BAM i + 2 reuses
        its slot.  The next BAMs' bytes are read into pinned memory on another thread.  Accumulation stays in the given
        order (the same history as one process_bam per BAM); a BAM the device path declines takes the records plan in
        its turn."""
        from concurrent.futures import ThreadPoolExecutor
        prm = self.pileup_params
        nt = max(1, prm.n_threads // 2)

        def read(path):
            bam = AlignmentFile(path)
            if contig not in bam.references:
                bam.close()
                raise ValueError(f"invalid contig `{contig}`")
            return bam, bam.bam_map(nt)

        def finish(job):
            slot, bam, fut = job
            try:
                batch = fut.result()
                with self._lock:
                    if batch.n_cols == 0:
                        batch.close()
                        return
                    self._use_reference(referenceIndex)
                    self.engine.bam_slot(slot)
                    if self.engine.bam_accumulate(batch):
                        self._inflight.append((self.engine.input_ticket(), batch))
                        self._drain(keep=2)
                        self._batch_contig.append(referenceIndex)
                        return
                    batch.close()
                    log.info("device BAM plan declined: %s", self.engine.bam_fallback)
                self._accumulate_plan(bam.pileup_records(contig, prm), referenceIndex)
            finally:
                bam.close()

        self.last_bam_path = "device"
        with ThreadPoolExecutor(1) as io, ThreadPoolExecutor(1) as planner:
            maps = [io.submit(read, p) for p in paths[:2]]
            pending = None
            done = False
            try:
                for i in range(len(paths)):
                    bam, bmap = maps[i].result()
                    maps[i] = None
                    if i + 2 < len(paths):
                        maps.append(io.submit(read, paths[i + 2]))
                    slot = i & 1
                    # BAM i + 1's compressed bytes start up into the other slot (its previous BAM, i - 1, has been
                    # opened; its fill reads only the inflated records), overlapping BAM i's inflate
                    if i + 1 < len(paths):
                        nb, nm = maps[i + 1].result()
                        self.engine.bam_upload(nm, slot ^ 1)
                    plan = None
                    try:
                        with self._lock:
                            self.engine.bam_slot(slot)
                            n = self.engine.bam_open(bmap, bam.tid(contig), prm)
                            if n is not None and self.gpu_plan:
                                # htslib's depth cap / mate pairing on the GPU (spg_bam_plan_build): nothing comes down
                                plan = self.engine.bam_plan_build(prm.max_depth, prm.ignore_overlaps)
                            reads = self.engine.bam_reads(n) if n is not None and plan is None else None
                    finally:
                        bmap.close()
                    if pending is not None:           # BAM i - 1: planned on the worker while BAM i opened
                        job, pending = pending, None
                        finish(job)
                    if plan is not None:              # in order, after BAM i - 1
                        ok = True
                        with self._lock:
                            if plan.n_cols:
                                self._use_reference(referenceIndex)
                                self.engine.bam_slot(slot)
                                ok = self.engine.bam_accumulate_planned(plan)
                                if ok:
                                    self._batch_contig.append(referenceIndex)
                        if not ok:
                            log.info("device BAM plan declined %s: %s", paths[i], self.engine.bam_fallback)
                            try:
                                self._accumulate_plan(bam.pileup_records(contig, prm), referenceIndex)
                            finally:
                                bam.close()
                        else:
                            bam.close()
                        continue
                    if reads is None:                 # declined: the records plan, in order
                        log.info("device BAM path declined %s: %s", paths[i], self.engine.bam_fallback)
                        try:
                            self._accumulate_plan(bam.pileup_records(contig, prm), referenceIndex)
                        finally:
                            bam.close()
                        continue
                    pending = (slot, bam, planner.submit(bam.pileup_fields, contig, reads, prm))
                if pending is not None:
                    job, pending = pending, None
                    finish(job)
                done = True
            finally:
                if pending is not None:
                    pending[2].cancel()
                    pending[1].close()
                if not done:
                    # an error: an upload of the next BAM may still read its pinned map — wait for it and drop it from
                    # its slot (spg_bam_release) before the maps are closed
                    try:
                        self.engine.bam_release()
                    except Exception as e:          # (never masks the error that got us here)
                        log.warning("spg_bam_release after an error: %s", e)
                for f in maps:
                    if f is not None:
                        try:
                            b, m = f.result()
                            m.close()
                            b.close()
                        except Exception:
                            pass
                with self._lock:
                    self.engine.bam_slot(0)

    def _accumulate_plan(self, batch, referenceIndex):
        with self._lock:
            if batch.is_records:
                if batch.n_cols == 0:
                    batch.close()
                    return
                self._use_reference(referenceIndex)
                self.engine.accumulate_bam_records(batch)
                # the plan's pinned buffers are copied on the engine's copy stream: keep them until that copy lands
                self._inflight.append((self.engine.input_ticket(), batch))
                self._drain(keep=2)
                self._batch_contig.append(referenceIndex)
                return
            if batch.n_cols == 0:
                batch.fill()
                batch.close()
                return
            codes, quals, offs = self._ingest.buffers(batch.n_entries, batch.n_cols)
            batch.fill(codes, quals)
            offs[:batch.n_cols + 1] = batch.offsets
            E = batch.n_entries
            self._use_reference(referenceIndex)
            self.engine.accumulate(batch.pos_begin, offs[:batch.n_cols + 1], codes[:E], quals[:E], trusted=True)
            self._ingest.enqueued()
            self._batch_contig.append(referenceIndex)
        batch.close()

    def prepare_variants(self) -> List[Variant]:
        """:120-231"""
        with self._lock:
            self._drain()
            self.engine.finalize()
            return self.engine.variants()

    # -- checkpoint ---------------------------------------------------------------------------
    def create_checkpoint(self, filename):
        """:40-45 — the accumulated batches (exact engine state) as numpy .npz files.  Like the reference's
        pickled `memory`, which holds only the base qualities that passed the filter (:96-103), each batch keeps
        only its entries with q >= minBaseQuality — plus, for a column whose every entry fails it, its first
        entry, so that the position's first visit (:77-85) survives the round trip.  The compaction runs on the GPU
        (spg_history_copy_compact): only the kept bytes cross PCIe, no per-entry host arrays.

        Incremental: `filename` is a small manifest (FASTA names, contig of every batch, the shard files); the
        batches live in shard files beside it (`spgck-<memory token>-<first batch>-<count>.npz`), which belong to
        this memory, not to one manifest name.  vc_queue.py:134-144 writes a checkpoint after every BAM, under a new
        name per BAM (`<temp dir>/<bam name><ext>`): each call writes only the batches accumulated since this
        memory's previous checkpoint in that directory (whatever its name), and its manifest lists the earlier
        shards too — O(new entries) per BAM, and every manifest stays a complete, loadable state.  A reset or a load
        starts a new memory (a new token: its first checkpoint writes every batch once).  Manifests are replaced
        atomically after their shards are on disk; shards an overwritten manifest listed are removed when no
        manifest in the directory lists them any more."""
        log.info("Creating checkpoint %s", filename)
        with self._lock:
            self.flush_checkpoints()                     # (the previous one's files are complete from here on)
            n = self.engine.history_count()
            names = list(self.fastaFile.references)
            d = os.path.dirname(os.path.abspath(filename))
            shards = []                                  # this memory's shard chain in d, while its files exist
            for sh in self._ck_chain.get(d, []):
                if not os.path.exists(os.path.join(d, sh[0])):
                    break
                shards.append(sh)
            first = sum(k for _, _, k in shards)
            if first > n:
                shards, first = [], 0
            self._ck_bytes = 0
            path, batches, behind = None, None, False
            if first < n:
                shard = f"spgck-{self._ck_token[:16]}-{first}-{n - first}.spgck"
                path = os.path.join(d, shard)
                # a single-device engine packs the kept entries one byte each on the GPU (A/C/G/T with q < 63; the rest
                # as exceptions): half the bytes down and on disk
                if isinstance(self.engine, PileupEngine):
                    if self.checkpoint_write_behind:
                        batches = self.engine.copy_history_packed(first, self.minBaseQuality)
                        behind = batches is not None
                    if batches is None:
                        batches = self.engine.iter_history_packed(first, self.minBaseQuality)
                else:
                    batches = self.engine.iter_history(first, min_bq=self.minBaseQuality)
                shards.append((shard, first, n - first))
            elif self.checkpoint_write_behind:
                behind = True
            self._ck_chain[d] = list(shards)
            man = dict(format=np.int64(2), token=np.array(self._ck_token),
                       contig=np.array(self._batch_contig, np.int64), names=np.array(names),
                       min_base_quality=np.int64(self.minBaseQuality),
                       shard_files=np.array([s for s, _, _ in shards] or [""]),
                       shard_ranges=np.array([[a, k] for _, a, k in shards], np.int64).reshape(-1, 2))

            def write():
                size = _write_shard(path, batches) if path is not None else 0
                old = _read_manifest(filename)
                tmp = filename + ".tmp"
                with open(tmp, "wb") as f:
                    np.savez(f, **man)
                os.replace(tmp, filename)
                if old is not None:
                    gone = {s for s, _, _ in old["shards"]} - {s for s, _, _ in shards}
                    if gone:
                        _remove_unlisted(d, gone)
                return size

            if behind:
                if self._ck_pool is None:
                    from concurrent.futures import ThreadPoolExecutor
                    self._ck_pool = ThreadPoolExecutor(1, thread_name_prefix="spg-checkpoint")
                self._ck_job = self._ck_pool.submit(write)
                key, job = os.path.abspath(filename), self._ck_job
                with _PENDING_LOCK:
                    _PENDING[key] = job

                def _done(_f, key=key, job=job):
                    with _PENDING_LOCK:
                        if _PENDING.get(key) is job:
                            del _PENDING[key]
                job.add_done_callback(_done)
            else:
                self._ck_bytes = write()

    def flush_checkpoints(self):
        """Wait for the write-behind checkpoint in flight (create_checkpoint) and raise the error it met, if any."""
        with self._lock:
            job, self._ck_job = self._ck_job, None
            if job is not None:
                self._ck_bytes = job.result()

    @property
    def last_checkpoint_bytes(self) -> int:
        """Shard bytes the last create_checkpoint wrote (waits for a write-behind checkpoint)."""
        self.flush_checkpoints()
        return self._ck_bytes

    def load_checkpoint(self, filename):
        """:47-52 — replaces memory with the checkpoint's (replays its batches).  Reads the incremental
        manifest format and the single-file format of earlier versions."""
        log.info("Loading checkpoint %s", filename)
        self.flush_checkpoints()
        with _PENDING_LOCK:                              # another caller's write-behind checkpoint of this file
            job = _PENDING.get(os.path.abspath(filename))
        if job is not None:
            job.result()
        man = _read_manifest(filename)
        if man is not None:
            if man["names"] != self.fastaFile.references:
                raise ValueError("checkpoint was made with a different reference FASTA")
            # shards keep only the entries that passed the writer's minBaseQuality (plus first-visit markers):
            # another threshold would silently change depths and calls
            if man["min_base_quality"] != self.minBaseQuality:
                raise ValueError(f"checkpoint was made with minBaseQuality {man['min_base_quality']}, "
                                 f"this caller uses {self.minBaseQuality}")
            d = os.path.dirname(os.path.abspath(filename))
            contig, batches = man["contig"], []
            for s, a, k in man["shards"]:
                if s.endswith(".spgck"):
                    got = _read_shard(os.path.join(d, s))
                    if len(got) != k:
                        raise ValueError(f"checkpoint shard {s}: {len(got)} batches, the manifest lists {k}")
                    batches += got
                    continue
                with np.load(os.path.join(d, s), allow_pickle=False) as z:
                    batches += [(int(z[f"b{i}_pos"]), z[f"b{i}_off"], z[f"b{i}_codes"], z[f"b{i}_quals"])
                                for i in range(k)]
        else:
            with np.load(filename, allow_pickle=False) as z:
                contig = z["contig"].tolist()
                names = z["names"].tolist()
                if names != self.fastaFile.references:
                    raise ValueError("checkpoint was made with a different reference FASTA")
                batches = [(int(z[f"b{i}_pos"]), z[f"b{i}_off"], z[f"b{i}_codes"], z[f"b{i}_quals"])
                           for i in range(len(contig))]
        if len(batches) != len(contig):
            raise ValueError(f"checkpoint {filename}: {len(batches)} batches for {len(contig)} contig entries")
        with self._lock:
            self.reset_memory()
            for ci, (pb, off, codes, quals) in zip(contig, batches):
                self._use_reference(ci)
                self.engine.accumulate(pb, off, codes, quals)
                self._batch_contig.append(ci)

    # -- output ------------------------------------------------------------------------------
    def write_vcf(self, outputVfc: str):
        """:233-297"""
        print("VFC output", outputVfc)
        variants = self.prepare_variants()
        records = sorted(variants, key=lambda v: (v["start"], v["info"]["SCORE"]))
        contigs = [(r, self.fastaFile.get_reference_length(r)) for r in self.fastaFile.references]
        try:
            import pysam  # noqa: F401
        except ImportError:
            pysam = None
        if pysam is not None:
            _write_vcf_pysam(pysam, outputVfc, contigs, records)
        else:
            write_vcf_text(outputVfc, contigs, records)


INFO_META = [
    ("DP", "1", "Integer", "Total Depth"),
    ("AD", "1", "Integer", "Allele Depth"),
    ("GL", "1", "Float", "Genotype likelihoods comprised of comma separated floating point log10-scaled "
                         "likelihoods for all possible genotypes given the set of alleles defined in the REF "
                         "and ALT fields"),
    ("PL", "1", "Integer", "The phred-scaled genotype likelihoods rounded to the closest integer (and otherwise "
                           "defined precisely as the GL field)"),
    ("SCORE", "1", "Float", "Custom scoring function"),
]


_PENDING_LOCK = threading.Lock()
_PENDING: Dict[str, object] = {}      # manifest path -> the write-behind checkpoint (Future) that last wrote it


def _read_manifest(filename):
    """The incremental checkpoint manifest at `filename` (create_checkpoint), or None when the file is absent,
    unreadable or in the single-file format."""
    try:
        with np.load(filename, allow_pickle=False) as z:
            if "format" not in z.files or int(z["format"]) != 2:
                return None
            files = [str(x) for x in z["shard_files"].tolist()]
            rng = z["shard_ranges"].reshape(-1, 2).tolist()
            shards = [(f, int(a), int(k)) for f, (a, k) in zip(files, rng)]
            contig = z["contig"].tolist()
            return {"token": str(z["token"]), "names": [str(x) for x in z["names"].tolist()],
                    "contig": contig, "n": len(contig), "min_base_quality": int(z["min_base_quality"]),
                    "shards": shards}
    except (OSError, ValueError, KeyError, TypeError, AttributeError):   # (a plain .npy holds an ndarray, not a zip)
        return None


def _is_bgzf(path: str) -> bool:
    with open(path, "rb") as f:
        return f.read(2) == b"\x1f\x8b"


_SHARD_MAGIC, _SHARD_END = b"SPGCKv1\0", b"SPGCKEND"


_SHARD_SPLIT = 64 << 20      # arrays of at least this many bytes are written in _SHARD_PARTS files at once
_SHARD_PARTS = 4


def _shard_side(path: str, j: int) -> str:
    return f"{path}.x{j}"


def _write_shard(path: str, batches) -> int:
    """A checkpoint shard: each batch's arrays written as they come (64-B aligned raw arrays, no per-array CRC or copy —
    np.savez's zip CRC and buffer copies took most of a 10,000x BAM's checkpoint), then a JSON index and its offset.  A
    batch is (pos, offsets, codes, quals) or a dict of named arrays (engine.iter_history_packed: offsets, the packed
    bytes and the exception list).  An array of >= _SHARD_SPLIT bytes goes out in _SHARD_PARTS pieces at once: the
    first in this file, the others in side files <path>.x<j> written by helper threads (the page-cache copy into one
    file is serial in the kernel; parallel writes into one file measured no faster); its index entry lists them.  Side
    files are complete before <path>.tmp is renamed to <path>.  Returns the bytes written (main + side files)."""
    import json
    import struct
    from concurrent.futures import ThreadPoolExecutor
    index, sides, jobs = [], [], []

    def write_side(j, view):
        with open(_shard_side(path, j) + ".tmp", "wb") as g:
            g.write(view)
        os.replace(_shard_side(path, j) + ".tmp", _shard_side(path, j))

    with ThreadPoolExecutor(_SHARD_PARTS - 1) as ex, open(path + ".tmp", "wb") as f:
        f.write(_SHARD_MAGIC)
        for b in batches:
            if not isinstance(b, dict):
                b = {"pos": b[0], "off": b[1], "codes": b[2], "quals": b[3]}
            ent = {"pos": int(b["pos"])}
            for name, a in b.items():
                if name == "pos":
                    continue
                a = np.ascontiguousarray(a)
                pad = (-f.tell()) % 64
                if pad:
                    f.write(b"\0" * pad)
                ent[name] = [f.tell(), int(a.size), a.dtype.str]
                mv = memoryview(a).cast("B")
                if mv.nbytes >= _SHARD_SPLIT:
                    step = ((mv.nbytes + _SHARD_PARTS - 1) // _SHARD_PARTS + 4095) // 4096 * 4096
                    parts = []
                    for k in range(1, _SHARD_PARTS):
                        lo, hi = min(mv.nbytes, k * step), min(mv.nbytes, (k + 1) * step)
                        j = len(sides)
                        sides.append(hi - lo)
                        parts.append([os.path.basename(_shard_side(path, j)), hi - lo])
                        jobs.append(ex.submit(write_side, j, mv[lo:hi]))
                    ent[name] += [min(step, mv.nbytes), parts]
                    f.write(mv[:min(step, mv.nbytes)])
                else:
                    f.write(mv)
            # the side files of this batch are written before the next batch is asked for: a generator may hand out
            # views of one reused buffer (engine.iter_history_packed's pinned staging), which its next batch overwrites
            for j in jobs:
                j.result()
            jobs.clear()
            index.append(ent)
        at = f.tell()
        f.write(json.dumps(index).encode())
        f.write(struct.pack("<Q", at) + _SHARD_END)
        size = f.tell()
    os.replace(path + ".tmp", path)
    return size + sum(sides)


_PACKED_CODE = np.array([1, 2, 4, 8], np.uint8)


def _read_shard(path: str):
    """[(pos_begin, offsets, codes, quals)] of a _write_shard file (no code from the file is executed: raw arrays of
    the dtypes its index names, u64 / u8 only); packed batches are decoded (byte >> 6 -> A/C/G/T, byte & 63 -> q, then
    the exceptions)."""
    import json
    import struct
    with open(path, "rb") as f:
        if f.read(8) != _SHARD_MAGIC:
            raise ValueError(f"{path}: not a checkpoint shard")
        f.seek(-16, os.SEEK_END)
        at, end = struct.unpack("<Q8s", f.read(16))
        if end != _SHARD_END:
            raise ValueError(f"{path}: truncated checkpoint shard")
        size = f.tell()
        f.seek(at)
        index = json.loads(f.read(size - 16 - at))
        out = []
        for ent in index:
            arrs = {}
            for name in ("off", "codes", "quals", "packed", "xi", "xc", "xq"):
                if name not in ent:
                    continue
                pos, n, dt = ent[name][:3]
                if dt not in ("<u8", "|u1"):
                    raise ValueError(f"{path}: unexpected dtype {dt}")
                f.seek(pos)
                if len(ent[name]) == 3:
                    arrs[name] = np.fromfile(f, dtype=np.dtype(dt), count=n)
                    continue
                # an array in pieces (_write_shard): this file's, then the side files' (names checked: <shard>.x<j>)
                a = np.empty(n, np.dtype(dt))
                buf = memoryview(a).cast("B")
                n0, parts = int(ent[name][3]), ent[name][4]
                if n0 + sum(int(k) for _, k in parts) != buf.nbytes:
                    raise ValueError(f"{path}: array pieces do not add up")
                if f.readinto(buf[:n0]) != n0:
                    raise ValueError(f"{path}: truncated checkpoint shard")
                o = n0
                for side, k in parts:
                    if not (isinstance(side, str) and side.startswith(os.path.basename(path) + ".x") and "/" not in side):
                        raise ValueError(f"{path}: bad side file name {side!r}")
                    with open(os.path.join(os.path.dirname(path), side), "rb") as g:
                        if g.readinto(buf[o:o + int(k)]) != int(k):
                            raise ValueError(f"{path}: truncated side file {side}")
                    o += int(k)
                arrs[name] = a
            if "packed" in arrs:
                pk = arrs["packed"]
                codes, quals = _PACKED_CODE[pk >> 6], pk & np.uint8(63)
                xi = arrs["xi"].astype(np.int64)
                if len(xi) and (xi.min() < 0 or xi.max() >= len(pk)):
                    raise ValueError(f"{path}: exception index out of range")
                codes[xi] = arrs["xc"]
                quals[xi] = arrs["xq"]
            else:
                codes, quals = arrs["codes"], arrs["quals"]
            out.append((int(ent["pos"]), arrs["off"], codes, quals))
    return out


def _remove_unlisted(d: str, files):
    """Delete the shard files among `files` that no manifest in directory d lists (several manifests share one
    memory's shards).  Runs only when a manifest was overwritten with a different shard list (a reset, a load, or a
    foreign memory under the same name), so its O(files in d) scan is off the per-BAM path."""
    listed = set()
    with os.scandir(d) as it:
        for ent in it:
            if not ent.is_file() or ent.name.startswith("spgck-") or ent.name.endswith(".tmp"):
                continue
            m = _read_manifest(ent.path)
            if m is not None:
                listed.update(s for s, _, _ in m["shards"])
    for s in set(files) - listed:
        for p in [os.path.join(d, s)] + [os.path.join(d, x) for x in os.listdir(d) if x.startswith(s + ".x")]:
            try:
                os.remove(p)
            except OSError:
                pass


def _hval(v: str) -> str:
    """htslib header value quoting as pysam's add_meta does it (quote when it holds ' ;,"\\t<>')."""
    return f'"{v}"' if any(ch in v for ch in ' ;,"\t<>') else v


def _f32(x) -> str:
    """A Float field as htslib prints it: stored as float32, printed with %g."""
    return "%g" % float(np.float32(x))


def write_vcf_text(path: str, contigs, records: List[Variant]):
    """The VCF text pysam.VariantFile(mode='w') writes for the reference's header (:235-278)."""
    out = ["##fileformat=VCFv4.2", '##FILTER=<ID=PASS,Description="All filters passed">']
    for i, n, t, d in INFO_META:
        out.append(f"##INFO=<ID={i},Number={n},Type={t},Description={_hval(d)}>")
    for name, length in contigs:
        out.append(f"##contig=<ID={name},length={length}>")
    out.append("#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO")
    chrom = contigs[0][0] if contigs else "."          # new_record() without contig -> rid 0
    for v in records:
        info = v["info"]
        fields = []
        for key, _, typ, _ in INFO_META:
            if key not in info:
                continue
            val = info[key]
            fields.append(f"{key}={int(val)}" if typ == "Integer" else f"{key}={_f32(val)}")
        out.append("\t".join([chrom, str(v["start"] + 1), ".", v["alleles"][0], v["alleles"][1], _f32(v["qual"]), ".",
                              ";".join(fields)]))
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")


def _write_vcf_pysam(pysam, path, contigs, records):
    h = pysam.VariantHeader()
    for i, n, t, d in INFO_META:
        h.add_meta("INFO", items=[("ID", i), ("Number", int(n)), ("Type", t), ("Description", d)])
    for name, length in contigs:
        h.contigs.add(name, length)
    vf = pysam.VariantFile(path, mode="w", header=h)
    for v in records:
        vf.write(vf.new_record(start=v["start"], stop=v["stop"], alleles=v["alleles"], qual=v["qual"], info=v["info"]))
    vf.close()
