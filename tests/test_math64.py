"""The f64 softplus / log / sigmoid of the Adam objective (csrc/pmg_math64.h) against the
long-double C library: the stop rule compares consecutive losses to 1e-6 relative, so the
loss terms must stay within a few f64 ulps (fit_tuning_helper.py:63-81 evaluates them in
f64 through jax.nn.softplus and xlogy)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.mark.skipif(shutil.which('g++') is None, reason="needs g++")
def test_math64_accuracy(tmp_path):
    exe = tmp_path / 'math64_check'
    subprocess.run(['g++', '-O2', '-std=c++17', '-I', os.path.join(ROOT, 'poor_man_gplvm_amd', 'csrc'),
                    os.path.join(HERE, 'native', 'math64_check.cpp'), '-o', str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    softplus, logf, sigmoid, exp_, log_, t_softplus, t_logf, t_sigmoid_rel, t_log, t_exp = map(float, out)
    # series forms (f64 ulps; log(f) in eps relative to max(1, |log f|))
    assert softplus <= 4.0
    assert logf <= 6.0
    assert sigmoid <= 4.0
    assert exp_ <= 2.0
    assert log_ <= 3.0
    # table forms used by k_adam: softplus and its log to a few f64 ulps, the sigmoid to f32
    assert t_softplus <= 5.0
    assert t_logf <= 7.0
    assert t_log <= 3.0
    assert t_sigmoid_rel <= 3e-7
    assert t_exp <= 3.0
