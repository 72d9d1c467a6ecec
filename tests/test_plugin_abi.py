"""Grok's plugin ABI (libgrok_plugin.so, include/grk_plugin_abi.h): loaded the
way Grok's host loads it (dlopen, minpf_post_load_plugin with a
platform-services table, then the plugin_* symbols by name; grok.cpp:810-861,
minpf_plugin.h:37-57).  CPU: registration, exports, return conventions and
plugin_init == false without a GPU; gpu: plugin_init brings up the MI355X
context."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

LIB = os.path.join(ROOT, "grokimagecompression_amd", "lib", "libgrok_plugin.so")
HDR = os.path.join(ROOT, "include", "grk_plugin_abi.h")

# names Grok's host dlsyms (grok.cpp:810-823) and the debug hooks
HOST_NAMES = ["plugin_get_debug_state", "plugin_init", "plugin_encode", "plugin_batch_encode",
              "plugin_stop_batch_encode", "plugin_is_batch_complete", "plugin_decode",
              "plugin_init_batch_decode", "plugin_batch_decode", "plugin_stop_batch_decode",
              "minpf_post_load_plugin"]


class Version(ctypes.Structure):
    _fields_ = [("major", ctypes.c_int32), ("minor", ctypes.c_int32)]


CREATE = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p)
DESTROY = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p)


class RegisterParams(ctypes.Structure):
    _fields_ = [("version", Version), ("createFunc", CREATE), ("destroyFunc", DESTROY)]


REGISTER = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_char_p, ctypes.POINTER(RegisterParams))
INVOKE = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_char_p, ctypes.c_void_p)


class Services(ctypes.Structure):
    _fields_ = [("version", Version), ("registerObject", REGISTER), ("invokeService", INVOKE)]


class InitInfo(ctypes.Structure):
    _fields_ = [("deviceId", ctypes.c_int32), ("verbose", ctypes.c_bool)]


EXIT = ctypes.CFUNCTYPE(ctypes.c_int32)


def _load():
    import grokimagecompression_amd as grk
    grk.lib()  # torch + the HIP runtime first, as for every grkgpu user
    if not os.path.exists(LIB):
        grk.build()
    L = ctypes.CDLL(LIB)
    L.minpf_post_load_plugin.restype = ctypes.c_void_p
    L.minpf_post_load_plugin.argtypes = [ctypes.c_char_p, ctypes.POINTER(Services)]
    L.plugin_init.restype = ctypes.c_bool
    L.plugin_init.argtypes = [InitInfo]
    L.plugin_get_debug_state.restype = ctypes.c_uint32
    L.plugin_is_batch_complete.restype = ctypes.c_bool
    for f in ("plugin_encode", "plugin_decode", "plugin_batch_decode"):
        getattr(L, f).restype = ctypes.c_int32
    L.plugin_batch_encode.restype = ctypes.c_int32
    L.plugin_init_batch_decode.restype = ctypes.c_int32
    return L


def _register(L, rc=0):
    seen = []

    def reg(node, params):
        p = params.contents
        seen.append((node.decode(), p.version.major, p.version.minor, bool(p.createFunc), bool(p.destroyFunc)))
        return rc

    cb_reg, cb_inv = REGISTER(reg), INVOKE(lambda n, p: 0)
    svc = Services(Version(1, 0), cb_reg, cb_inv)
    ex = L.minpf_post_load_plugin(b"/plugins", ctypes.byref(svc))
    return ex, seen


def test_exports_header_and_host_names():
    L = _load()
    declared = set(re.findall(r"^[a-z_0-9 ]+\**\s*((?:plugin|minpf)_[a-z_]+)\s*\(", open(HDR).read(), re.M))
    assert {"plugin_encode", "plugin_decode", "minpf_post_load_plugin"} <= declared
    for name in sorted(declared | set(HOST_NAMES)):
        assert hasattr(L, name), name


def test_registration_and_conventions():
    L = _load()
    ex, seen = _register(L)
    assert seen == [("GrokMI355X", 1, 0, True, True)]
    assert ex
    ex2, _ = _register(L, rc=-1)   # host refused the object -> no exit function
    assert not ex2
    assert L.plugin_get_debug_state() == 0
    assert L.plugin_encode(None, None) == -1
    assert L.plugin_batch_encode(b"in", b"out", None, None) == -1
    assert L.plugin_decode(None, None) == -1
    # 0 = no batch set up: the reference host starts a batch decode only on a
    # non-zero return (grk_decompress.cpp:1242-1245)
    assert L.plugin_init_batch_decode(b"in", b"out", None, None) == 0
    assert L.plugin_batch_decode() == -1
    assert L.plugin_is_batch_complete()
    assert EXIT(ex)() == 0


def test_init_false_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    L = _load()
    assert not L.plugin_init(InitInfo(0, False))


@pytest.mark.gpu
def test_init_brings_up_gpu_context():
    L = _load()
    ex, seen = _register(L)
    assert L.plugin_init(InitInfo(0, False))
    assert L.plugin_init(InitInfo(0, True))      # idempotent
    assert EXIT(ex)() == 0                       # exit releases the context
