"""ctypes mirror of include/tbf.h (the drop-in C-ABI)."""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

# TBF_LIB overrides the library path (build variants for A/B measurements)
LIB_PATH = Path(os.environ.get("TBF_LIB", Path(__file__).resolve().parent / "libtbf.so"))

_fp = C.POINTER(C.c_float)
_dp = C.POINTER(C.c_double)
_u32p = C.POINTER(C.c_uint32)


# the render kernels of one launch chunk, in stream order (tbf_debug_kernel_times)
STAGES = ("k_tonegen", "k_mixpre", "k_rv_pre", "k_rv_core", "k_rv_post", "k_whirl")


class TbfError(RuntimeError):
    pass


class _Config(C.Structure):
    _fields_ = [("sample_rate", C.c_double), ("device", C.c_int32), ("chain_mode", C.c_uint32),
                ("debug_flags", C.c_uint32), ("reserved", C.c_uint32 * 3)]


# tbf_engine_config.debug_flags / tbf_error_flags bits (include/tbf.h)
DEBUG_FORCE_SERIAL = 1
PATH_VIB_SERIAL, PATH_WH_ANGLE, PATH_WH_MOTION, PATH_RV_PHASE, PATH_RV_WINDOW = 1, 2, 4, 8, 16


# every symbol include/tbf.h declares, with its ctypes signature
SIGNATURES = {
    "tbf_abi_version": (C.c_int, []),
    "tbf_last_error": (C.c_char_p, []),
    "tbf_engine_create": (C.c_int, [C.POINTER(_Config), C.POINTER(C.c_void_p)]),
    "tbf_engine_destroy": (C.c_int, [C.c_void_p]),
    "tbf_template_create": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, _u32p]),
    "tbf_templates_create": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, _u32p, _u32p]),
    "tbf_instances_add": (C.c_int, [C.c_void_p, C.c_uint32, _u32p, _u32p, _u32p]),
    "tbf_instance_count": (C.c_uint32, [C.c_void_p]),
    "tbf_instance_retune": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32]),
    "tbf_note": (C.c_int, [C.c_void_p, C.c_uint32, C.c_int32, C.c_int32]),
    "tbf_set_param": (C.c_int, [C.c_void_p, C.c_uint32, C.c_int32, C.c_double]),
    "tbf_render": (C.c_int, [C.c_void_p, C.c_uint32, _fp, _fp, C.c_uint64]),
    "tbf_render_device": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]),
    "tbf_synth_sound": (C.c_int, [C.c_void_p, C.c_uint32, _fp, _fp, C.c_uint64]),
    "tbf_synchronize": (C.c_int, [C.c_void_p]),
    "tbf_error_flags": (C.c_int, [C.c_void_p, _u32p]),
    "tbf_template_bank": (C.c_int, [C.c_void_p, C.c_uint32, _fp, C.c_uint64, _u32p]),
    "tbf_midi_control": (C.c_int, [C.c_void_p, C.c_uint32, C.c_char_p, C.c_int32]),
    "tbf_config_set": (C.c_int, [C.c_void_p, C.c_char_p, C.c_char_p]),
    "tbf_config_parse": (C.c_int, [C.c_void_p, C.c_char_p]),
    "tbf_program_parse": (C.c_int, [C.c_void_p, C.c_char_p]),
    "tbf_program_install": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32]),
    "tbf_program_name": (C.c_int, [C.c_void_p, C.c_uint32, C.c_char_p, C.c_uint32]),
    "tbf_midi_control_id": (C.c_int, [C.c_char_p]),
    "tbf_set_steady_chunk": (C.c_int, [C.c_void_p, C.c_uint32]),
    "tbf_render_events": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                    C.c_uint64, C.c_void_p]),
}

# tbf_event kinds (include/tbf.h)
EV_NOTE, EV_PARAM, EV_CONTROL, EV_PROGRAM = 0, 1, 2, 3
EVENT_DTYPE = np.dtype([("block", "<u4"), ("inst", "<u4"), ("kind", "<i4"), ("id", "<i4"), ("value", "<f8")])

_lib = None


def load_library():
    """Load the in-tree libtbf.so; fails loudly when it has not been built."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise TbfError(f"{LIB_PATH} not built -- run __graft_entry__.build() or `make -C tunebfree_amd`")
        lib = C.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        _lib = lib
    return _lib


def _check(rc):
    if rc < 0:
        raise TbfError(f"tbf error {rc}: {load_library().tbf_last_error().decode(errors='replace')}")
    return rc


class Engine:
    """A batch of organ instances on one GPU (one engine per device / rank)."""

    def __init__(self, sample_rate=48000.0, device=0, chain=0, debug_flags=0):
        lib = load_library()
        cfg = _Config(float(sample_rate), int(device), int(chain), int(debug_flags))
        h = C.c_void_p()
        _check(lib.tbf_engine_create(C.byref(cfg), C.byref(h)))
        self._lib, self._h = lib, h
        self.sample_rate, self.device = sample_rate, device

    def close(self):
        if getattr(self, "_h", None):
            self._lib.tbf_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def config_set(self, key, value):
        """One cfg key (tbf_config_set): 0 applied, 1 not a key of this path."""
        return _check(self._lib.tbf_config_set(self._h, str(key).encode(), str(value).encode()))

    def config(self, items):
        """Several cfg keys, a dict or (key, value) pairs, in order."""
        for k, v in (items.items() if isinstance(items, dict) else items):
            self.config_set(k, v)

    def config_parse(self, text):
        """A cfg file's text; returns the number of keys applied."""
        return _check(self._lib.tbf_config_parse(self._h, text.encode()))

    def layout(self):
        """The cfg-derived layout (tbf_debug_layout): compact whirl ring window, the
        geometry's largest write-ahead, reverb slab length."""
        f = self._lib.tbf_debug_layout
        f.restype = C.c_int
        f.argtypes = [C.c_void_p, _u32p, _fp, _u32p]
        w, a, s = C.c_uint32(), C.c_float(), C.c_uint32()
        _check(f(self._h, C.byref(w), C.byref(a), C.byref(s)))
        return {"wring_len": w.value, "max_ahead": a.value, "slab_len": s.value}

    def front_chunks(self):
        """tbf_debug_front_chunks: chunks with events stepped by (the device's, the host's) front end"""
        f = self._lib.tbf_debug_front_chunks
        f.restype, f.argtypes = C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]
        d, h = C.c_uint64(), C.c_uint64()
        _check(f(self._h, C.byref(d), C.byref(h)))
        return d.value, h.value

    def set_steady_chunk(self, blocks):
        """tbf_set_steady_chunk: the longest chunk without control deltas (64..2048 blocks),
        which bounds the stage buffers; returns the value in effect."""
        return _check(self._lib.tbf_set_steady_chunk(self._h, int(blocks)))

    def chunks(self):
        """Blocks per render chunk (tbf_debug_chunks): (with control deltas, without)."""
        f = self._lib.tbf_debug_chunks
        f.restype = C.c_int
        f.argtypes = [C.c_void_p, _u32p, _u32p]
        d, s = C.c_uint32(), C.c_uint32()
        _check(f(self._h, C.byref(d), C.byref(s)))
        return d.value, s.value

    def template(self, mts128=None, ratio9=None, seed=1):
        m = None if mts128 is None else np.ascontiguousarray(mts128, dtype=np.float64)
        r = None if ratio9 is None else np.ascontiguousarray(ratio9, dtype=np.float64)
        out = C.c_uint32()
        _check(self._lib.tbf_template_create(self._h, None if m is None else m.ctypes.data,
                                             None if r is None else r.ctypes.data, int(seed), C.byref(out)))
        return out.value

    def templates(self, seeds, mts128=None, ratio9=None):
        """n templates built on the device (tbf_templates_create): mts128 (n, 128) or
        None, ratio9 (n, 9) or None; returns the template ids."""
        sd = np.ascontiguousarray(seeds, dtype=np.uint32).reshape(-1)
        n = len(sd)
        m = None if mts128 is None else np.ascontiguousarray(mts128, dtype=np.float64).reshape(n, 128)
        r = None if ratio9 is None else np.ascontiguousarray(ratio9, dtype=np.float64).reshape(n, 9)
        ids = np.zeros(n, np.uint32)
        _check(self._lib.tbf_templates_create(self._h, n, None if m is None else m.ctypes.data,
                                              None if r is None else r.ctypes.data,
                                              sd.ctypes.data_as(_u32p), ids.ctypes.data_as(_u32p)))
        return [int(x) for x in ids]

    def template_bank(self, tpl):
        lens = np.zeros(256, np.uint32)
        n = _check(self._lib.tbf_template_bank(self._h, int(tpl), None, 0, lens.ctypes.data_as(_u32p)))
        out = np.zeros(n, np.float32)
        _check(self._lib.tbf_template_bank(self._h, int(tpl), out.ctypes.data_as(_fp), n, None))
        return out, lens

    def retune(self, inst, tpl_id):
        """tbf_instance_retune: the CLAP reinitToneGen on another template, from the next block"""
        _check(self._lib.tbf_instance_retune(self._h, int(inst), int(tpl_id)))

    def add_instances(self, tpl_ids, seeds):
        t = np.ascontiguousarray(tpl_ids, dtype=np.uint32)
        s = np.ascontiguousarray(seeds, dtype=np.uint32)
        assert t.shape == s.shape
        first = C.c_uint32()
        _check(self._lib.tbf_instances_add(self._h, len(t), t.ctypes.data_as(_u32p), s.ctypes.data_as(_u32p),
                                           C.byref(first)))
        return first.value

    @property
    def n_instances(self):
        return self._lib.tbf_instance_count(self._h)

    def note(self, inst, key, on):
        _check(self._lib.tbf_note(self._h, int(inst), int(key), int(on)))

    def set_param(self, inst, pid, value):
        _check(self._lib.tbf_set_param(self._h, int(inst), int(pid), float(value)))

    def render(self, nblocks):
        """Synchronous render into host arrays, shape [n_instances, nblocks*128]."""
        n = self.n_instances
        L = np.zeros((n, nblocks * 128), np.float32)
        R = np.zeros((n, nblocks * 128), np.float32)
        _check(self._lib.tbf_render(self._h, int(nblocks), L.ctypes.data_as(_fp), R.ctypes.data_as(_fp),
                                    nblocks * 128))
        return L, R

    def render_device(self, nblocks, outL_ptr, outR_ptr, stride, stream=None):
        """Enqueue a render into device memory (e.g. torch tensor data_ptr())."""
        _check(self._lib.tbf_render_device(self._h, int(nblocks), C.c_void_p(int(outL_ptr)),
                                           C.c_void_p(int(outR_ptr)), int(stride),
                                           None if stream is None else C.c_void_p(int(stream))))

    def synth_sound(self, nframes):
        n = self.n_instances
        L = np.zeros((n, nframes), np.float32)
        R = np.zeros((n, nframes), np.float32)
        _check(self._lib.tbf_synth_sound(self._h, int(nframes), L.ctypes.data_as(_fp), R.ctypes.data_as(_fp),
                                         nframes))
        return L, R

    def midi_control(self, inst, fn, value):
        """callMIDIControlFunction (src/midi.cpp:535): True if the name is a hot-path control."""
        return _check(self._lib.tbf_midi_control(self._h, int(inst), fn.encode(), int(value))) == 0

    def program_parse(self, text):
        """Load programme definitions in the reference's .pgm syntax; returns programmes in use."""
        return _check(self._lib.tbf_program_parse(self._h, text.encode()))

    def program_install(self, inst, pc):
        """installProgram (src/program.cpp:735) for MIDI program change pc on one instance."""
        _check(self._lib.tbf_program_install(self._h, int(inst), int(pc)))

    def program_name(self, pc):
        buf = C.create_string_buffer(64)
        return buf.value.decode() if _check(self._lib.tbf_program_name(self._h, int(pc), buf, 64)) else None

    def control_id(self, fn):
        return self._lib.tbf_midi_control_id(fn.encode())

    def events(self, rows):
        """Pack (block, inst, kind, id, value) rows into the tbf_event array, stably sorted
        by block."""
        a = np.array([tuple(r) for r in rows], dtype=EVENT_DTYPE)
        return a[np.argsort(a["block"], kind="stable")] if len(a) else a

    def render_events_device(self, nblocks, events, outL_ptr, outR_ptr, stride, stream=None):
        """tbf_render_events: enqueue a render of nblocks with scheduled events into device
        memory (e.g. torch tensor data_ptr())."""
        ev = np.ascontiguousarray(events, dtype=EVENT_DTYPE)
        _check(self._lib.tbf_render_events(self._h, int(nblocks), ev.ctypes.data if len(ev) else None, len(ev),
                                           C.c_void_p(int(outL_ptr)), C.c_void_p(int(outR_ptr)), int(stride),
                                           None if stream is None else C.c_void_p(int(stream))))

    def synchronize(self):
        _check(self._lib.tbf_synchronize(self._h))

    def kernel_times(self, enable=None):
        """Per-stage HIP-event timing (tbf_debug_kernel_times): enable=True/False switches
        recording ("serial": with cross-chunk pipelining off, each kernel alone); with no
        argument returns {stage: (ms_total, launches)} since the last call."""
        fn = self._lib.tbf_debug_kernel_times
        fn.restype, fn.argtypes = C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]
        if enable is not None:
            _check(fn(self._h, -1 if not enable else (2 if enable == "serial" else 1), None, None))
            return None
        ms = np.zeros(8, np.float64)  # room for any build's stage count (A/B against older builds)
        cnt = np.zeros(8, np.uint32)
        _check(fn(self._h, 0, ms.ctypes.data, cnt.ctypes.data))
        return {k: (float(ms[i]), int(cnt[i])) for i, k in enumerate(STAGES)}

    def host_time(self, reset=True):
        """tbf_debug_host_time: (ms of host control stepping, blocks) since the last reset"""
        fn = self._lib.tbf_debug_host_time
        fn.restype, fn.argtypes = C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]
        ms, nb = C.c_double(), C.c_uint64()
        _check(fn(self._h, 1 if reset else 0, C.byref(ms), C.byref(nb)))
        return ms.value, nb.value

    def debug_reverb_phase(self, inst, ch, line, value):
        """test hook (tbf_debug_reverb_phase): set a reverb vibrato phase, from the next block"""
        fn = self._lib.tbf_debug_reverb_phase
        fn.restype, fn.argtypes = C.c_int, [C.c_void_p, C.c_uint32, C.c_int32, C.c_int32, C.c_double]
        _check(fn(self._h, int(inst), int(ch), int(line), float(value)))

    def error_flags(self):
        f = C.c_uint32()
        _check(self._lib.tbf_error_flags(self._h, C.byref(f)))
        return f.value
