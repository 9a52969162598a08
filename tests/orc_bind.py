"""ctypes bindings for the CPU oracle (oracle/liborc.so) and, where present, the
reference-compiled checker (oracle/_ref/libtbfref.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
ORC_SO = ROOT / "oracle" / "liborc.so"
REF_SO = ROOT / "oracle" / "_ref" / "libtbfref.so"
PIN_SO = ROOT / "oracle" / "_ref" / "libtbfpin.so"
WPIN_SO = ROOT / "oracle" / "_ref" / "libtbfwpin.so"
# the same reference TUs built with the reference's release flags (common.mak:16-18):
# the CPU baseline's timing build (bench.py), never a parity checker
REF_FAST_SO = ROOT / "oracle" / "_ref" / "fast" / "libtbfref.so"

_fp = C.POINTER(C.c_float)
_dp = C.POINTER(C.c_double)
_u32p = C.POINTER(C.c_uint32)


def _f(a):
    return None if a is None else a.ctypes.data_as(_fp)


def load_oracle():
    if not ORC_SO.exists():
        raise FileNotFoundError(f"{ORC_SO} missing -- run `make -C oracle`")
    lib = C.CDLL(str(ORC_SO))
    lib.orc_template_new.restype = C.c_void_p
    lib.orc_template_new.argtypes = [C.c_double, C.c_void_p, C.c_void_p, C.c_uint]
    lib.orc_template_free.argtypes = [C.c_void_p]
    lib.orc_template_dump.argtypes = [C.c_void_p, C.c_char_p]
    lib.orc_template_bank_size.restype = C.c_size_t
    lib.orc_template_bank_size.argtypes = [C.c_void_p]
    lib.orc_template_bank.argtypes = [C.c_void_p, _fp, _u32p]
    lib.orc_template_envs.argtypes = [C.c_void_p, _fp, _fp, _fp]
    lib.orc_fitwave.restype = C.c_size_t
    lib.orc_fitwave.argtypes = [C.c_double, C.c_double, C.c_int, C.c_int, C.c_double]
    lib.orc_get_frequencies.argtypes = [_dp, C.c_void_p]
    lib.orc_infer_scale_size.argtypes = [_dp, C.POINTER(C.c_int), C.POINTER(C.c_float)]
    lib.orc_srand.argtypes = [C.c_void_p, C.c_uint]
    lib.orc_rand_next.restype = C.c_int32
    lib.orc_rand_next.argtypes = [C.c_void_p]
    lib.orc_inst_new.restype = C.c_void_p
    lib.orc_inst_new.argtypes = [C.c_void_p, C.c_uint]
    lib.orc_inst_free.argtypes = [C.c_void_p]
    lib.orc_note.argtypes = [C.c_void_p, C.c_int, C.c_int]
    lib.orc_set_param.argtypes = [C.c_void_p, C.c_int, C.c_double]
    lib.orc_set_chain.argtypes = [C.c_void_p, C.c_int]
    lib.orc_control.restype = C.c_int
    lib.orc_control.argtypes = [C.c_void_p, C.c_char_p, C.c_int]
    lib.orc_render.argtypes = [C.c_void_p, C.c_int, _fp, _fp, _fp, _fp, _fp]
    lib.orc_whirl_fields.restype = C.c_int
    lib.orc_whirl_fields.argtypes = [C.c_void_p, _dp]
    lib.orc_cfg_size.restype = C.c_size_t
    lib.orc_cfg_default.argtypes = [C.c_void_p]
    lib.orc_cfg_set.restype = C.c_int
    lib.orc_cfg_set.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p]
    lib.orc_template_new_cfg.restype = C.c_void_p
    lib.orc_template_new_cfg.argtypes = [C.c_double, C.c_void_p, C.c_void_p, C.c_uint, C.c_void_p]
    lib.orc_inst_new_cfg.restype = C.c_void_p
    lib.orc_inst_new_cfg.argtypes = [C.c_void_p, C.c_uint, C.c_void_p]
    lib.orc_inst_retune.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    for pre in ("orc",):
        getattr(lib, f"{pre}_whirl_new").restype = C.c_void_p
        getattr(lib, f"{pre}_whirl_new").argtypes = [C.c_double]
        getattr(lib, f"{pre}_whirl_rev_option").argtypes = [C.c_void_p, C.c_int]
        getattr(lib, f"{pre}_whirl_proc3").argtypes = [C.c_void_p, _fp, _fp, _fp, C.c_int]
        getattr(lib, f"{pre}_whirl_free").argtypes = [C.c_void_p]
        getattr(lib, f"{pre}_reverb_new").restype = C.c_void_p
        getattr(lib, f"{pre}_reverb_new").argtypes = [C.c_double, C.c_uint]
        getattr(lib, f"{pre}_reverb_set_mix").argtypes = [C.c_void_p, C.c_float]
        getattr(lib, f"{pre}_reverb_proc").argtypes = [C.c_void_p, _fp, _fp, C.c_int]
        getattr(lib, f"{pre}_reverb_free").argtypes = [C.c_void_p]
        getattr(lib, f"{pre}_preamp_new").restype = C.c_void_p
        getattr(lib, f"{pre}_preamp_new").argtypes = [C.c_double, C.c_uint]
        getattr(lib, f"{pre}_preamp_set").argtypes = [C.c_void_p, C.c_int, C.c_float]
        getattr(lib, f"{pre}_preamp_proc").argtypes = [C.c_void_p, _fp, _fp, C.c_int]
        getattr(lib, f"{pre}_preamp_free").argtypes = [C.c_void_p]
    return lib


def load_ref(fast=False):
    """The reference-compiled checker (strict IEEE build); None when not built.  fast=True:
    the release-flag build for timing (falls back to the strict one when absent)."""
    path = REF_FAST_SO if fast and REF_FAST_SO.exists() else REF_SO
    if not path.exists():
        return None
    lib = C.CDLL(str(path))
    lib.ref_inst_new.restype = C.c_void_p
    lib.ref_inst_new.argtypes = [C.c_void_p, C.c_uint]
    lib.ref_inst_free.argtypes = [C.c_void_p]
    lib.ref_inst_new_cfg.restype = C.c_void_p
    lib.ref_inst_new_cfg.argtypes = [C.c_void_p, C.c_uint, C.c_void_p]
    lib.ref_inst_retune.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lib.ref_note.argtypes = [C.c_void_p, C.c_int, C.c_int]
    lib.ref_set_param.argtypes = [C.c_void_p, C.c_int, C.c_double]
    lib.ref_set_chain.argtypes = [C.c_void_p, C.c_int]
    lib.ref_control.restype = C.c_int
    lib.ref_control.argtypes = [C.c_void_p, C.c_char_p, C.c_int]
    lib.ref_render.argtypes = [C.c_void_p, C.c_int, _fp, _fp, _fp, _fp, _fp]
    lib.ref_whirl_new.restype = C.c_void_p
    lib.ref_whirl_new.argtypes = [C.c_double]
    lib.ref_whirl_rev_option.argtypes = [C.c_void_p, C.c_int]
    lib.ref_whirl_proc3.argtypes = [C.c_void_p, _fp, _fp, _fp, C.c_int]
    lib.ref_whirl_free.argtypes = [C.c_void_p]
    lib.ref_reverb_new.restype = C.c_void_p
    lib.ref_reverb_new.argtypes = [C.c_double, C.c_uint]
    lib.ref_reverb_set_mix.argtypes = [C.c_void_p, C.c_float]
    lib.ref_reverb_proc.argtypes = [C.c_void_p, _fp, _fp, C.c_int]
    lib.ref_reverb_free.argtypes = [C.c_void_p]
    lib.ref_preamp_new.restype = C.c_void_p
    lib.ref_preamp_new.argtypes = [C.c_double, C.c_uint]
    lib.ref_preamp_set.argtypes = [C.c_void_p, C.c_int, C.c_float]
    lib.ref_preamp_proc.argtypes = [C.c_void_p, _fp, _fp, C.c_int]
    lib.ref_preamp_free.argtypes = [C.c_void_p]
    return lib


def load_pin():
    """The template-pin harness (oracle/ref_tpl_pin.cpp: src/tonegen.cpp's own static
    table builders); None when not built (e.g. on the GPU box)."""
    if not PIN_SO.exists():
        return None
    lib = C.CDLL(str(PIN_SO))
    lib.refpin_template.restype = C.c_long
    lib.refpin_template.argtypes = [C.c_double, _dp, C.c_void_p, C.c_uint, _fp, C.c_uint64, _u32p, _dp, _fp, _fp,
                                    _fp]
    lib.refpin_template_cfg.restype = C.c_long
    lib.refpin_template_cfg.argtypes = [C.c_double, _dp, C.c_void_p, C.c_uint, C.c_void_p, _fp, C.c_uint64, _u32p,
                                        _dp, _fp, _fp, _fp]
    lib.refpin_template_full.restype = C.c_long
    lib.refpin_template_full.argtypes = [C.c_double, _dp, C.c_void_p, C.c_uint, C.c_void_p, _fp, C.c_uint64, _u32p,
                                         _dp, _fp, _fp, _fp, _u32p, C.c_void_p, C.c_void_p, _fp, C.c_uint32]
    return lib


CONTRIB_CAP = 1 << 17


def contrib_blob(n, wheel, bus, level):
    """The play matrix (keyContrib of keys 0..383) as one byte string: entries per key,
    then wheel / bus / level of all entries in key order."""
    t = int(np.sum(n))
    return np.frombuffer(np.asarray(n, np.uint32).tobytes() + np.asarray(wheel[:t], np.int16).tobytes() +
                         np.asarray(bus[:t], np.int16).tobytes() + np.asarray(level[:t], np.float32).tobytes(),
                         np.uint8)


def contrib_from(fn):
    """contrib_blob of a per-key exporter fn(key, wheel_ptr, bus_ptr, level_ptr, cap) -> count
    (orc_template_contrib / tbf_debug_contrib)."""
    cap = 4096
    n = np.zeros(384, np.uint32)
    W, B, L = [], [], []
    w, b, lv = np.zeros(cap, np.int16), np.zeros(cap, np.int16), np.zeros(cap, np.float32)
    for k in range(384):
        c = fn(k, w.ctypes.data, b.ctypes.data, lv.ctypes.data, cap)
        assert 0 <= c <= cap, (k, c)
        n[k] = c
        W.append(w[:c].copy()); B.append(b[:c].copy()); L.append(lv[:c].copy())
    return contrib_blob(n, np.concatenate(W), np.concatenate(B), np.concatenate(L))


def pin_template(pin, orc, sr, mts128, seed, cfg=None):
    """Wave bank, lengths, wheel frequencies, envelopes and key-compression table built by
    the reference's own initOscillators / initKeyCompTable / initEnvelopes (with the
    template keys of an oracle Cfg record, set through the reference's own setters)."""
    f300 = np.zeros(300, np.float64)
    m = None if mts128 is None else np.ascontiguousarray(mts128, np.float64)
    orc.orc_get_frequencies(f300.ctypes.data_as(_dp), None if m is None else m.ctypes.data)
    cp = None if cfg is None else cfg.ptr
    n = pin.refpin_template_full(float(sr), f300.ctypes.data_as(_dp), None, int(seed), cp, None, 0, None, None, None,
                                 None, None, None, None, None, None, 0)
    bank = np.zeros(n, np.float32)
    lens = np.zeros(256, np.uint32)
    wf = np.zeros(256, np.float64)
    a = np.zeros((9, 128), np.float32)
    r = np.zeros((9, 128), np.float32)
    k = np.zeros(128, np.float32)
    cn = np.zeros(384, np.uint32)
    cw, cb, cl = np.zeros(CONTRIB_CAP, np.int16), np.zeros(CONTRIB_CAP, np.int16), np.zeros(CONTRIB_CAP, np.float32)
    pin.refpin_template_full(float(sr), f300.ctypes.data_as(_dp), None, int(seed), cp, _f(bank), n,
                             lens.ctypes.data_as(_u32p), wf.ctypes.data_as(_dp), _f(a), _f(r), _f(k),
                             cn.ctypes.data_as(_u32p), cw.ctypes.data, cb.ctypes.data, _f(cl), CONTRIB_CAP)
    assert int(cn.sum()) <= CONTRIB_CAP
    return {"bank": bank, "lens": lens, "wfreq": wf, "attack": a, "release": r, "keycomp": k,
            "contrib": contrib_blob(cn, cw, cb, cl)}


class Cfg:
    """An oracle cfg record (orc_cfg): the reference's defaults plus key=value lines."""

    def __init__(self, lib, items=()):
        self.lib = lib
        self.buf = C.create_string_buffer(lib.orc_cfg_size())
        lib.orc_cfg_default(self.buf)
        for k, v in (items.items() if isinstance(items, dict) else items):
            self.set(k, v)

    def set(self, key, value):
        return self.lib.orc_cfg_set(self.buf, str(key).encode(), str(value).encode())

    @property
    def ptr(self):
        return C.cast(self.buf, C.c_void_p)


class Template:
    """Tonegen template (wave bank + play matrix + envelopes) built by the oracle."""

    def __init__(self, lib, sr=48000.0, mts128=None, ratio9=None, seed=1, cfg=None):
        self.lib = lib
        self._mts = None if mts128 is None else np.ascontiguousarray(mts128, dtype=np.float64)
        self._rat = None if ratio9 is None else np.ascontiguousarray(ratio9, dtype=np.float64)
        self.cfg = cfg
        self.ptr = lib.orc_template_new_cfg(
            float(sr),
            None if self._mts is None else self._mts.ctypes.data,
            None if self._rat is None else self._rat.ctypes.data,
            int(seed),
            None if cfg is None else cfg.ptr,
        )
        self.sr = sr

    def bank(self):
        n = self.lib.orc_template_bank_size(self.ptr)
        out = np.zeros(n, np.float32)
        lens = np.zeros(256, np.uint32)
        self.lib.orc_template_bank(self.ptr, _f(out), lens.ctypes.data_as(_u32p))
        return out, lens

    def envs(self):
        a = np.zeros((9, 128), np.float32)
        r = np.zeros((9, 128), np.float32)
        k = np.zeros(128, np.float32)
        self.lib.orc_template_envs(self.ptr, _f(a), _f(r), _f(k))
        return a, r, k

    def contrib(self):
        """contrib_blob of the oracle's play matrix"""
        self.lib.orc_template_contrib.restype = C.c_int
        self.lib.orc_template_contrib.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        return contrib_from(lambda k, w, b, lv, cap: self.lib.orc_template_contrib(self.ptr, k, w, b, lv, cap))

    def dump(self, d):
        return self.lib.orc_template_dump(self.ptr, str(d).encode())

    def __del__(self):
        try:
            self.lib.orc_template_free(self.ptr)
        except Exception:
            pass


class Chain:
    """One organ instance driven through either the oracle or the reference checker."""

    def __init__(self, lib, tpl: Template, seed: int, ref: bool = False, cfg=None):
        self.lib, self.ref = lib, ref
        p = "ref" if ref else "orc"
        self._new = getattr(lib, f"{p}_inst_new_cfg")
        self._note = getattr(lib, f"{p}_note")
        self._param = getattr(lib, f"{p}_set_param")
        self._chain = getattr(lib, f"{p}_set_chain")
        self._render = getattr(lib, f"{p}_render")
        self._free = getattr(lib, f"{p}_inst_free")
        self._retune = getattr(lib, f"{p}_inst_retune")
        self._control = getattr(lib, f"{p}_control")
        self.cfg = cfg if cfg is not None else tpl.cfg
        self.ptr = self._new(tpl.ptr, int(seed), None if self.cfg is None else self.cfg.ptr)
        self.tpl = tpl

    def note(self, key, on):
        self._note(self.ptr, int(key), int(on))

    def param(self, pid, value):
        self._param(self.ptr, int(pid), float(value))

    def chain(self, mode):
        self._chain(self.ptr, int(mode))

    def control(self, name, value):
        """a whirl MIDI control function by name (value 0..127), from the next block"""
        if self._control(self.ptr, name.encode(), int(value)) != 0:
            raise ValueError(f"not a whirl control function: {name}")

    def retune(self, tpl: Template):
        """the CLAP reinitToneGen on another template, from the next block"""
        self._retune(self.ptr, tpl.ptr, None if self.cfg is None else self.cfg.ptr)
        self.tpl = tpl  # the oracle's tonegen points into it

    def render(self, nblocks, stages=False):
        n = nblocks * 128
        L = np.zeros(n, np.float32)
        R = np.zeros(n, np.float32)
        if stages:
            A = np.zeros(n, np.float32)
            B = np.zeros(n, np.float32)
            Cc = np.zeros(n, np.float32)
            self._render(self.ptr, nblocks, _f(L), _f(R), _f(A), _f(B), _f(Cc))
            return L, R, A, B, Cc
        self._render(self.ptr, nblocks, _f(L), _f(R), None, None, None)
        return L, R

    def __del__(self):
        try:
            self._free(self.ptr)
        except Exception:
            pass


def fptr(a):
    return _f(a)


def load_wpin():
    """The whirl-setter pin harness (oracle/ref_whirl_pin.cpp: src/whirl.cpp's own static
    MIDI control setters, built without the CLAP define); None when not built."""
    if not WPIN_SO.exists():
        return None
    lib = C.CDLL(str(WPIN_SO))
    lib.wpin_new.restype = C.c_void_p
    lib.wpin_new.argtypes = [C.c_double]
    lib.wpin_free.argtypes = [C.c_void_p]
    lib.wpin_control.restype = C.c_int
    lib.wpin_control.argtypes = [C.c_void_p, C.c_char_p, C.c_int]
    lib.wpin_fields.restype = C.c_int
    lib.wpin_fields.argtypes = [C.c_void_p, _dp]
    return lib
