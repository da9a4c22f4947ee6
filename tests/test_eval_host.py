"""Host logic of the whole-scan corrector (CPU): the restated patchly squeeze-mode grid."""


def test_grid_origins_squeeze():
    from cgan3d_amd.eval.CCTAContrastCorrector import grid_origins
    o = grid_origins((40, 32, 45), (16, 16, 16))
    assert sorted({a for a, _, _ in o}) == [0, 16, 24] and sorted({b for _, b, _ in o}) == [0, 16]
    assert sorted({c for _, _, c in o}) == [0, 16, 29] and len(o) == 18
