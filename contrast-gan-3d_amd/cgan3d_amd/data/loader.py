"""Pinned-host -> HBM patch loader: drop-in for the reference's 3-D training loaders.

Replaces ``CCTADataLoader`` + the batchgenerators augmenter wrapped around it
(``contrast_gan_3D/data/CCTADataLoader.py:14-108``, built by ``trainer/utils.py:44-107``):
``next(loader)`` returns the reference's batch dict ``{"data", "seg", "name", "path"}`` with
``data`` a float32 [B,1,W,H,D] patch batch and ``seg`` the boolean centre-line mask, already in
HBM.

Per batch:
* host worker threads copy each sample's crop straight out of the memory-mapped
  ``<patient>.npy`` volume (4-D ``[W,H,D,(HU,label)]``, ``data/utils.py:34-54``) into a pinned
  staging slot.  The crop follows ``generate_one`` (``CCTADataLoader.py:88-104``): dims smaller
  than the patch are zero-padded symmetrically (batchgenerators ``pad_nd_image``:
  below = diff // 2, above = the rest), the others are cropped at a uniformly random offset
  (``crop(..., crop_type="random")``), drawn here from the loader's ``numpy.random.Generator``;
* the worker that filled a slot also queues its asynchronous host-to-device (SDMA) copy on the copy
  stream (``ops.pooled_stream(dev, "copy")``, shared by the loaders of a device), so the transfer's
  host-side cost stays off the trainer's thread; ``cgan3d_unpack_patches`` then de-interleaves and
  scales the batch on the GPU ((HU - shift) / factor, ``FactorZeroCenterScaler``,
  ``data/Scaler.py:37-45``).  ``zero_copy=True``: the slots are mapped into the device
  (``cgan3d_host_alloc``) and one ``cgan3d_unpack_patches_ex`` launch reads them over PCIe instead;
* ``depth`` batches are in flight: host workers read ahead, and ``next()`` also issues the device
  work of the following batches whose host reads are done, each ordered only after the consumers of
  its slot's previous batch, so batch j+1 crosses PCIe while the step on batch j runs.  A returned
  batch's tensors live in a ring slot and are overwritten ``depth`` batches later (the Trainer
  consumes each batch within its step).

* augmentation (optional ``transform``, ``data/augment.py``: batchgenerators'
  ``SpatialTransform_2`` as ``basic_conf.py:87-113`` configures it, and ``MirrorTransform`` after it
  as ``conf_2D.py:36-43`` does — one transform or a list run in order): the per-sample parameters
  and the elastic noise fields are drawn on the host with the crop boxes, under the loader's lock
  from its one generator (a single random stream, as batchgenerators draws per batch); the host
  worker pins them for the async copy, and ``cgan3d_spatial_augment`` / ``cgan3d_mirror`` transform
  the unpacked batch on the loader stream.

2-D patches (``experiments/conf_2D.py``: a patch shape of two entries) follow
``CCTADataLoader.get_samplable_2D`` (``CCTADataLoader.py:50-70``): with probability 1/2 a patch
around a random centre-line point of the scan's ``<patient>_meta`` record (world -> image
coordinates, ``utils/geometry.py:21-26``; bounds ``get_patch_bounds``, ``:114-138``, with its
(y, x) argument order kept) in that point's slice, not cropped further; otherwise a random slice
of the scan, padded and randomly cropped like a 3-D patch.  ``data`` is then [B, 1, W, H].
"""
from __future__ import annotations

import threading
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import ops


def _scaler_params(scaler) -> Tuple[float, float]:
    """(shift, factor) of the reference's scalers: FactorZeroCenterScaler (shift, factor),
    ZeroCenterScaler (shift), or the identity default of CCTADataLoader (``lambda x: x``)."""
    if scaler is None:
        return 0.0, 1.0
    shift = getattr(scaler, "shift", None)
    if shift is not None:
        return float(shift), float(getattr(scaler, "factor", 1))
    probe = np.array([-1000.0, 0.0, 1234.0], dtype=np.float32)
    if np.array_equal(np.asarray(scaler(probe), dtype=np.float32), probe):
        return 0.0, 1.0
    raise TypeError("PatchLoader: scaler must be a (Factor)ZeroCenterScaler or the identity")


def crop_box(shape: Sequence[int], patch: Sequence[int], rng: np.random.Generator):
    """Per-dim (src_lo, dst_lo, length) of CCTADataLoader.generate_one's pad-then-random-crop:
    batchgenerators' ``pad_nd_image`` then ``crop(crop_type="random")``, whose
    ``get_lbs_for_random_crop`` draws ``randint(0, s - p)`` where s - p > 0 (the last offset is never
    drawn) and takes (s - p) // 2 otherwise (no draw)."""
    box = []
    for s, p in zip(shape, patch):
        if s < p:  # pad_nd_image: centred zero padding; the padded dim equals the patch (offset 0)
            box.append((0, (p - s) // 2, s))
        elif s > p:
            box.append((int(rng.integers(0, s - p)), 0, p))
        else:
            box.append((0, 0, p))
    return box


def read_crop(vol: np.ndarray, patch: Sequence[int], box, out: np.ndarray):
    """out[W,H,D,2] = zero-padded crop of vol[W,H,D,2] described by ``box``; a 2-D ``box`` =
    (z, ((src_lo, dst_lo, length) in W, in H)): out[W,H,2] from slice z."""
    if len(patch) == 2:
        z, ((sx, dx, lx), (sy, dy, ly)) = box
        if (dx, dy) != (0, 0) or (lx, ly) != tuple(patch):
            out.fill(0)
        out[dx:dx + lx, dy:dy + ly] = vol[sx:sx + lx, sy:sy + ly, z]
        return
    (sx, dx, lx), (sy, dy, ly), (sz, dz, lz) = box
    if (dx, dy, dz) != (0, 0, 0) or (lx, ly, lz) != tuple(patch):
        out.fill(0)
    out[dx:dx + lx, dy:dy + ly, dz:dz + lz] = vol[sx:sx + lx, sy:sy + ly, sz:sz + lz]


class _MetaUnpickler:
    """Restricted unpickling of the reference's ``_meta.pkl`` records (data/utils.py:48-54: a dict of
    numpy arrays, floats and a name): only builtin containers / scalars and numpy array / dtype /
    scalar reconstruction resolve; any other global (arbitrary code) raises UnpicklingError."""

    ALLOWED = {("builtins", n) for n in ("dict", "list", "tuple", "set", "frozenset", "str", "int", "float",
                                          "complex", "bool", "bytes", "bytearray", "slice", "range")}
    ALLOWED |= {(m, n) for m in ("numpy.core.multiarray", "numpy._core.multiarray")
                for n in ("_reconstruct", "scalar")}
    ALLOWED |= {("numpy", "ndarray"), ("numpy", "dtype"), ("collections", "OrderedDict")}

    @classmethod
    def load(cls, f):
        import pickle

        class _U(pickle.Unpickler):
            def find_class(self, module, name):
                if (module, name) in cls.ALLOWED or (module == "numpy" and name.endswith("DType")) or \
                        (module == "numpy.dtypes" and name.endswith("DType")):
                    return super().find_class(module, name)
                raise pickle.UnpicklingError(f"_meta.pkl: global {module}.{name} is not allowed")
        return _U(f).load()


def load_meta(path: str) -> dict:
    """A scan's metadata (offset, spacing, centerlines_world, name): ``<path>_meta.npz`` (numeric
    arrays, no code), else the reference's ``<path>_meta.pkl`` (data/utils.py:48-54 writes and reads
    it with pickle; the scan preparation of the user's own dataset) through a restricted unpickler
    that resolves numpy arrays and builtin containers only (_MetaUnpickler)."""
    npz = Path(path + "_meta.npz")
    if npz.is_file():
        with np.load(npz, allow_pickle=False) as z:
            meta = {k: z[k] for k in z.files}
        if "name" in meta:
            meta["name"] = str(meta["name"])
        return meta
    with open(path + "_meta.pkl", "rb") as f:
        return _MetaUnpickler.load(f)


def world_to_image(world, offset, spacing) -> np.ndarray:
    """utils/geometry.py:21-26: round((world - offset) / spacing) to int (3-D coordinates)."""
    world, offset, spacing = (np.asarray(a, dtype=np.float64) for a in (world, offset, spacing))
    if not (world.shape == offset.shape == spacing.shape == (3,)):
        raise ValueError("world_to_image: 3-D coordinates, offset and spacing")
    return ((world - offset) / spacing).round().astype(int)


def patch_bounds(target, source_shape, coords) -> np.ndarray:
    """utils/geometry.py:131-138 get_patch_bounds (with ensure_valid_bounds, :114-128): per dim
    [coord - half, coord + half + target % 2], shifted inside [0, size)."""
    target = np.array(target)
    half = np.where(target == -1, np.array(source_shape), target) // 2
    coords = np.asarray(coords)
    bbox = np.stack([coords - half, coords + half + target % 2], -1)
    for i, (t, size) in enumerate(zip(target, source_shape)):
        s, e = int(bbox[i, 0]), int(bbox[i, 1])
        if s < 0 and e > size:
            raise ValueError(f"patch_bounds: patch {int(t)} larger than the slice extent {size}")
        if s < 0:
            s, e = 0, int(t)
        if e > size:
            s, e = size - int(t), size
        if s < 0:  # the reference slices a shorter patch here and fails when it assembles the batch
            raise ValueError(f"patch_bounds: patch {int(t)} larger than the slice extent {size}")
        bbox[i] = (s, e)
    return bbox


def sample_2d(shape: Sequence[int], meta: dict, patch: Sequence[int], rng: np.random.Generator):
    """CCTADataLoader.get_samplable_2D + generate_one's pad-then-random-crop (CCTADataLoader.py:50-70,
    88-104) for a [W,H,D,2] scan: (z, W / H boxes of read_crop), drawing from ``rng`` in the
    reference's order: the branch, then the centre-line index or the slice, then (random slice)
    the crop offsets."""
    W, H, D = (int(x) for x in shape[:3])
    if rng.random() < 0.5:  # a patch around a random centre-line point, in its slice
        cl = np.asarray(meta["centerlines_world"])
        i = rng.integers(0, len(cl))
        x, y, z = world_to_image(cl[i, :3], meta["offset"], meta["spacing"])
        bb = patch_bounds(patch, (W, H), np.array([y, x]))  # the reference's (y, x) order
        if not -D <= z < D:
            raise IndexError(f"sample_2d: centre-line slice {z} outside the scan's {D} slices")
        box = tuple((int(lo), 0, int(hi - lo)) for lo, hi in bb)
        if tuple(b[2] for b in box) != tuple(patch):
            raise ValueError(f"sample_2d: centre-line patch {[b[2] for b in box]} != {tuple(patch)}")
        return int(z) % D, box
    z = int(rng.choice(D))
    return z, tuple(crop_box((W, H), patch, rng))


class PatchLoader:
    def __init__(self, data: List[str], patch_shape: Sequence[int], batch_size: int, rng: np.random.Generator,
                 scaler=None, infinite: bool = True, shuffle: bool = True, device=None, depth: int = 3,
                 num_threads: int = 4, seed_for_shuffle: Optional[int] = None, transform=None,
                 zero_copy: bool = False):
        if len(patch_shape) not in (2, 3):
            raise ValueError(f"PatchLoader: 2-D or 3-D patches, got {tuple(patch_shape)}")
        self.paths = [str(p) for p in data]
        self.patch = tuple(int(p) for p in patch_shape)
        self.planar = len(self.patch) == 2  # conf_2D: slices of the scans (sample_2d)
        self._metas = {}
        self.batch_size, self.rng, self.infinite, self.shuffle = batch_size, rng, infinite, shuffle
        self.shift, self.factor = _scaler_params(scaler)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.depth = max(2, depth)
        self._vols = {}
        probe = self._volume(self.paths[0])
        if probe.ndim != 4 or probe.shape[-1] != 2:
            raise ValueError(f"PatchLoader: expected [W,H,D,2] volumes, got {probe.shape}")
        # int16 scans travel as int16 (half the PCIe bytes); any other dtype is staged as float32,
        # which is what generate_one casts to before cropping
        self.dtype = torch.int16 if probe.dtype == np.int16 else torch.float32
        shp = (batch_size, *self.patch, 2)
        # zero_copy (round 5, off by default): the pinned slots are mapped into the device
        # (cgan3d_host_alloc) and the unpack kernel reads them over PCIe on a few blocks — one launch per
        # batch, no SDMA copy — but those blocks hold CUs for the transfer: the Trainer + loader step
        # measured 1.53 ms against 1.43 with the SDMA copies issued from the worker threads
        # (tools/h2d_probe.py); default: pinned slots, SDMA copy into a device slot, then the unpack
        self.zero_copy = bool(zero_copy)
        if self.zero_copy:
            self._mapped = [ops.MappedHost(shp, self.dtype) for _ in range(self.depth)]
            self._host = [m.tensor for m in self._mapped]
            self._raw = None
        else:
            self._host = [torch.empty(shp, dtype=self.dtype).pin_memory() for _ in range(self.depth)]
            self._raw = [torch.empty(shp, dtype=self.dtype, device=self.device) for _ in range(self.depth)]
        self._data = [torch.empty((batch_size, 1, *self.patch), device=self.device) for _ in range(self.depth)]
        self._seg = [torch.empty((batch_size, 1, *self.patch), dtype=torch.bool, device=self.device)
                     for _ in range(self.depth)]
        self._copied = [None] * self.depth  # HIP event: slot's H2D copy finished (host slot reusable)
        if transform is None:
            self.transforms = []
        else:
            self.transforms = list(transform) if isinstance(transform, (list, tuple)) else [transform]
        self.transform = self.transforms[0] if len(self.transforms) == 1 else (self.transforms or None)
        self._aug_ws = None
        for t in self.transforms:
            if not hasattr(t, "run"):
                raise TypeError(f"PatchLoader: transform {type(t).__name__} has no device implementation")
            if getattr(t, "patch_size", None) is None:
                t.patch_size = self.patch  # MirrorTransform: the patch it runs on
            if tuple(t.patch_size) != self.patch:
                raise ValueError(f"PatchLoader: transform patch {t.patch_size} != loader patch {self.patch}")
            if hasattr(t, "kernel_dims"):  # SpatialTransform_2: resampling workspace
                self._aug_ws = torch.empty(ops.augment_ws_floats(batch_size, t.kernel_dims, batch_size),
                                           device=self.device)
        if self.transforms:  # ping-pong with staging buffers so that the last transform writes the returned ones
            self._pre_data = [torch.empty_like(t) for t in self._data]
            self._pre_seg = [torch.empty_like(t) for t in self._seg]
        # one copy stream shared by every loader of the device, created with the engines' streams
        # (ops.pooled_stream): the engines' hardware-queue mapping does not depend on how many loaders exist
        self._stream = ops.pooled_stream(self.device, "copy")
        self._threads, self._pool = num_threads, None
        self._lock = threading.Lock()
        self._order_rng = np.random.default_rng(seed_for_shuffle)
        self._order, self._pos = [], 0
        self._pending, self._next_slot = {}, 0
        self.restart()

    # -- host side -----------------------------------------------------------------------------
    def _volume(self, path: str) -> np.ndarray:
        v = self._vols.get(path)
        if v is None:
            v = np.load(path + ".npy", mmap_mode="r")
            if getattr(self, "dtype", None) is torch.int16 and v.dtype != np.int16:
                raise TypeError(f"PatchLoader: {path}.npy is {v.dtype}, the other scans int16")
            self._vols[path] = v
        return v

    def _meta(self, path: str) -> dict:
        m = self._metas.get(path)
        if m is None:
            m = self._metas[path] = load_meta(path)
        return m

    def _indices(self) -> Optional[List[int]]:
        with self._lock:
            idx = []
            for _ in range(self.batch_size):
                if self._pos >= len(self._order):
                    if not self.infinite and self._order:
                        return None
                    self._order = list(range(len(self.paths)))
                    if self.shuffle:
                        self._order_rng.shuffle(self._order)
                    self._pos = 0
                idx.append(self._order[self._pos])
                self._pos += 1
            if self.planar:
                boxes = [sample_2d(self._volume(self.paths[i]).shape, self._meta(self.paths[i]), self.patch, self.rng)
                         for i in idx]
            else:
                boxes = [crop_box(self._volume(self.paths[i]).shape[:3], self.patch, self.rng) for i in idx]
            aug = None
            if self.transforms:  # drawn here, under the lock, from the loader's generator, in order
                aug = [t.draw(self.rng, self.batch_size) for t in self.transforms]
            return list(zip(idx, boxes)), aug

    def _fill(self, slot: int, picks, free):
        ev = self._copied[slot]
        if ev is not None:
            ev.synchronize()  # the previous H2D copy out of this pinned slot has finished
        host = self._host[slot].numpy()
        picks, aug = picks
        for b, (i, box) in enumerate(picks):
            read_crop(self._volume(self.paths[i]), self.patch, box, host[b])
        if aug is not None:  # small parameter / noise tensors, pinned by this worker for the async copy
            aug = [tuple(None if a is None else torch.from_numpy(np.ascontiguousarray(a)).pin_memory() for a in prm)
                   for prm in aug]
        if not self.zero_copy:
            # the SDMA copy is issued here, by the worker: a non-blocking copy of a pinned slot holds the
            # calling thread for about the transfer time (~0.3 ms per 4 MB, tools/h2d_probe.py), which on
            # the trainer's thread delayed the next step's launches.  Ordered after the consumers of the
            # slot's previous batch (``free``); the unpack the trainer's thread issues later on the same
            # stream follows it.
            with torch.cuda.device(self.device), torch.cuda.stream(self._stream):
                self._stream.wait_event(free)
                self._raw[slot].copy_(self._host[slot], non_blocking=True)
                done = torch.cuda.Event()
                done.record(self._stream)
                self._copied[slot] = done
        return picks, aug

    def _submit(self):
        picks = self._indices()
        if picks is None:
            return False
        slot = self._next_slot
        self._next_slot = (slot + 1) % self.depth
        self._pending[slot] = self._pool.submit(self._fill, slot, picks, self._free[slot])
        return True

    def restart(self):
        """Re-prime the pipeline (the Trainer calls this at the start of fit, Trainer.py:241-250)."""
        for f in self._pending.values():
            f.result()
        if self._pool is None:
            self._pool = ThreadPoolExecutor(max_workers=self._threads)
        self._pending, self._next_slot, self._pos, self._order = {}, 0, 0, []
        self._consume, self._ready, self._last = 0, {}, None
        # every slot's device buffers are free once the work enqueued so far has run
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._free = [ev] * self.depth
        self._aug_keep = [None] * self.depth
        for _ in range(self.depth - 1):
            if not self._submit():
                break

    def _finish(self):
        """Stop the host workers (Trainer end of fit); a later restart() starts them again."""
        if self._pool is not None:
            self._pool.shutdown(wait=True)
            self._pool, self._pending = None, {}

    # -- device side ---------------------------------------------------------------------------
    def __iter__(self):
        return self

    def _issue(self, slot: int):
        """Queue the slot's host-to-device copy, unpack and transforms on the copy stream, ordered
        only after the consumers of the batch that last used the slot's device buffers."""
        picks, aug = self._pending.pop(slot).result()  # (SDMA: the worker has queued the copy)
        with torch.cuda.stream(self._stream):
            bufs = [(self._data[slot], self._seg[slot]), (self._pre_data[slot], self._pre_seg[slot])] \
                if aug is not None else [(self._data[slot], self._seg[slot])]
            k = len(self.transforms) % 2 if aug is not None else 0  # the last transform ends in _data
            if self.zero_copy:
                self._stream.wait_event(self._free[slot])
                ops.unpack_patches_mapped(self._mapped[slot], *bufs[k], self.shift, self.factor)
                ev = torch.cuda.Event()
                ev.record(self._stream)
                self._copied[slot] = ev  # the host slot is free once this has run
            else:
                ops.unpack_patches(self._raw[slot], *bufs[k], self.shift, self.factor)
            if aug is not None:
                for t, prm in zip(self.transforms, aug):
                    dev = tuple(None if a is None else a.to(self.device, non_blocking=True) for a in prm)
                    t.run(dev, *bufs[k], *bufs[1 - k], ws=self._aug_ws)
                    k = 1 - k
                self._aug_keep[slot] = aug  # pinned sources alive until the slot is refilled
            ready = torch.cuda.Event()
            ready.record(self._stream)
        self._ready[slot] = (ready, picks)

    def __next__(self) -> dict:
        cur = torch.cuda.current_stream(self.device)
        if self._last is not None:
            # the batch handed out last has had its consumers enqueued by now: its slot is free once
            # they have run
            ev = torch.cuda.Event()
            ev.record(cur)
            self._free[self._last] = ev
        self._submit()  # keep depth - 1 batches ahead
        slot = self._consume
        if slot not in self._ready:
            if slot not in self._pending:
                raise StopIteration
            self._issue(slot)
        ready, picks = self._ready.pop(slot)
        self._consume = (slot + 1) % self.depth
        self._last = slot
        # the following batches whose host reads are done go over PCIe now, while the caller's step
        # on this batch runs (round 4 issued each copy only when its batch was asked for, behind the
        # whole previous step)
        nxt = self._consume
        for _ in range(self.depth - 1):
            fut = self._pending.get(nxt)
            if fut is None or not fut.done():
                break
            self._issue(nxt)
            nxt = (nxt + 1) % self.depth
        cur.wait_event(ready)
        names = [Path(self.paths[i]).name for i, _ in picks]
        return {"data": self._data[slot], "seg": self._seg[slot], "name": names,
                "path": [self.paths[i] for i, _ in picks]}

    def __len__(self):
        return len(self.paths)
