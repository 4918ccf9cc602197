"""The CPU baseline's JavaScript restatement (js/observerReplay.js) is a faithful observer: it
replays every reference-emitted golden log (tests/golden, produced by the transpiled reference)
to the reference's canonical state, errors included.  It is what bench.py times on the GPU box's
cores in place of the reference (which cannot travel), scaled by the calibration ratio r."""
import json
import os
import shutil
import subprocess

import pytest

from conftest import GOLDEN, GOLDEN_SETS, REPO, load_golden

NODE = shutil.which('node')
pytestmark = pytest.mark.skipif(not NODE, reason='node not installed')


@pytest.mark.parametrize('name', GOLDEN_SETS + ['errors'])
def test_restatement_replays_reference_goldens(name):
    _, exp = load_golden(name)
    out = subprocess.run([NODE, os.path.join(REPO, 'js', 'observerReplay.js'), 'state',
                          os.path.join(GOLDEN, name + '.mtlog')], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    got = [json.loads(x) for x in out.stdout.strip().split('\n')]
    assert len(got) == len(exp)
    for r, e in zip(got, exp):
        assert r['state'] == e['state'], (name, r['doc'])
        assert (r['err'] is None) == (e['err'] is None), (name, r['doc'])


def test_calibration_recorded():
    with open(os.path.join(REPO, 'profiles', 'r02_js_calibration.json')) as f:
        cal = json.load(f)
    assert 0.1 < cal['r'] < 10 and cal['threads'] >= 1 and cal['reference_ops_per_sec'] > 0
