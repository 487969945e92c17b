"""CPU: the row-program compiler (graph lowering, epilogue fusion, hand-derived backward, LDS
slot plan) executed by a numpy emulator of the kernel semantics, against the oracle's autodiff,
on every checkpoint signature of the reference."""
import numpy as np
import pytest

import hpe.compiler as C
import rowprog_emu as EMU
from oracle import keras_ref as K
from util import features, fixture, index, input_channels

IDS = sorted(r for r in index() if not r.startswith('reg1'))


def _flat(prog, w):
    p = np.zeros(prog.n_params)
    for k, (o, shp) in prog.param_index.items():
        p[o:o + int(np.prod(shp))] = w[k].ravel()
    p[prog.n_train:] = prog.consts
    return p


@pytest.mark.parametrize('rid', IDS)
def test_emulated_program_matches_oracle(rid):
    mc, w = fixture(rid)
    c = input_channels(mc)
    rng = np.random.default_rng(len(rid))
    n = 23
    x = rng.random((n, 1, 1, c)).astype(np.float32)
    y = (20 * rng.standard_normal((n, 3))).astype(np.float32)
    g = K.Graph(mc, w)
    ref = g.forward(x).detach().numpy().reshape(n, 3)
    pf = C.compile_graph(mc, w, 'fwd', fused=False)
    out = EMU.run(pf, _flat(pf, w), x.reshape(n, c))['out']
    np.testing.assert_allclose(out, ref, rtol=1e-5, atol=2e-5)
    try:
        pt = C.compile_graph(mc, w, 'train', fused=False)
    except ValueError as e:
        assert 'not on the hot path' in str(e) or 'does not fit' in str(e)
        return
    r = EMU.run(pt, _flat(pt, w), x.reshape(n, c), y_img=y.astype(np.float64), inv_count=1 / (n * 3),
                seed=77)
    grads, _, _ = K.gradients(g, x, y, drop_seed=77)
    for k, (o, shp) in pt.param_index.items():
        ref_g = grads[k].numpy().ravel() - 2 * g.l2[k] * g.params[k].numpy().ravel()
        got = r['grad'][o:o + int(np.prod(shp))]
        np.testing.assert_allclose(got, ref_g, rtol=1e-6, atol=1e-9 + 1e-6 * np.abs(ref_g).max(),
                                   err_msg=k)


def test_fused_recognition():
    kinds = {}
    for rid in IDS:
        mc, w = fixture(rid)
        kinds[rid] = C.compile_graph(mc, w, 'fwd').kind
    assert kinds['sqnu665j'] == 'mlp2' and kinds['stoqa9pt'] == 'mlp2'
    assert kinds['hrchr82r'] == 'chain' and kinds['ker7z9mv'] == 'generic'
    assert sum(v == 'mlp2' for v in kinds.values()) >= 10
    assert sum(v == 'chain' for v in kinds.values()) >= 20
    assert C.compile_graph(*fixture('hrchr82r'), 'train').kind == 'generic'   # chain is forward-only


def test_chain_words_emulated():
    """The KIND_CHAIN op words (field map of csrc/hpe_prog.h OP_CHAIN) reproduce the oracle."""
    n = 0
    for rid in IDS:
        mc, w = fixture(rid)
        prog = C.compile_graph(mc, w, 'fwd')
        if prog.kind != 'chain':
            continue
        n += 1
        c = input_channels(mc)
        x = features(64, c, seed=n)
        flat = np.zeros(prog.n_train, np.float32)
        for k, (o, shp) in prog.param_index.items():
            flat[o:o + int(np.prod(shp))] = np.asarray(w[k], np.float32).ravel()
        got = EMU.run_chain(prog, np.concatenate([flat, prog.consts]), x.reshape(-1, c))
        ref = K.Graph(mc, w).forward(x).detach().numpy().reshape(-1, 3)
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-4, err_msg=rid)
    assert n >= 20


def test_spatial_graph_rejects_non_row_local():
    mc, w = fixture('ker7z9mv')   # SE + MHA head: GAP / MHA need P == 1
    with pytest.raises(ValueError):
        C.compile_graph(mc, w, 'fwd', P=64, fused=False)


def test_slot_geometry_conflict_free():
    for c in (3, 8, 16, 32, 64, 88, 96, 128, 360, 512):
        cp, st = C.slot_geometry(c)
        assert cp % 8 == 0 and cp >= c and st % 4 == 0 and (st // 4) % 2 == 1
        banks = {((st * r) % 64) // 4 for r in range(16)}
        assert len(banks) == 16          # 16 rows x ds_read_b128: distinct bank quads


def test_large_programs_multi_pass_and_device_slots():
    """Round-2 geometry for graphs beyond one launch (csrc/hpe_rowprog.hip H_NPASS / H_GSLOTS): every
    dW block is owned by exactly one (pass, wave, accumulator) slot, passes are only used when one
    launch's 16 x 8 accumulators cannot hold the blocks, and slot plans beyond 160 KiB of LDS move to
    device scratch on the 16-wave kernel."""
    seen = {}
    for rid in ('66kjr5zw', '8equl7wt', 's25l3n04', '6togj6se', 'sqnu665j', 'hrchr82r'):
        mc, w = fixture(rid)
        p = C.compile_graph(mc, w, 'train', fused=False)
        wd = p.words
        npass, gs = int(wd[C.H_NPASS]), int(wd[C.H_GSLOTS])
        nw, acc = int(wd[C.H_NW]), int(wd[C.H_MAXACC])
        ndw = p.info['dw_blocks']
        blk = wd[int(wd[C.H_BLK_OFF]): int(wd[C.H_BLK_OFF]) + npass * nw * acc]
        used = [int(b) for b in blk if b >= 0]
        assert len(used) == ndw and len(set(used)) == ndw, rid
        assert npass == max(1, -(-ndw // (nw * acc))), rid
        if npass > 1:
            assert nw == 16 and acc == 8 and ndw > 128, rid
        if gs:
            assert nw == C.GS_NW, rid
        else:
            assert (int(wd[C.H_LDS_FLOATS]) + 32) * 4 <= 160 * 1024, rid
        seen[rid] = (npass, gs)
    assert seen['66kjr5zw'] == (3, 1) and seen['8equl7wt'] == (2, 0) and seen['6togj6se'] == (1, 1)
    assert seen['sqnu665j'][0] == 1 and seen['hrchr82r'] == (1, 0)
