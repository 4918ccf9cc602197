"""The C-ABI boundary (include/mtgpu.h) without a GPU: the library loads and exports every
symbol the header declares; host-side argument validation."""
import ctypes
import os
import re

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, 'include', 'mtgpu.h')


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r'^\s*(?:mt_status|const char\*)\s+(mt_\w+)\s*\(', src, re.M)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ('mt_engine_create', 'mt_docs_init', 'mt_submit', 'mt_batch_upload', 'mt_batch_apply', 'mt_sync',
              'mt_get_text', 'mt_get_state', 'mt_checksums', 'mt_doc_error', 'mt_engine_destroy'):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from fluidframework_amd import build
    build.build()
    lib = ctypes.CDLL(build.LIB)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    lib.mt_version.restype = ctypes.c_char_p
    assert b'gfx950' in lib.mt_version()


def test_op_record_layout_matches_header():
    from fluidframework_amd.oplog import OP_DTYPE
    assert OP_DTYPE.itemsize == 32
    assert [OP_DTYPE.fields[f][1] for f in OP_DTYPE.names] == [0, 4, 8, 12, 14, 15, 16, 20, 24, 28]


def test_engine_requires_the_hip_library(monkeypatch, tmp_path):
    from fluidframework_amd import engine
    monkeypatch.setattr(engine, 'LIB_PATH', str(tmp_path / 'missing.so'))
    monkeypatch.setattr(engine, '_lib', None)
    with pytest.raises(engine.MtError):
        engine.lib()
