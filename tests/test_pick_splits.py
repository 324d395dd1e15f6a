"""Split-KV choice of the flash-attention forward (ops/attention.py pick_splits) for the bench
configs' attention shapes: splits only where the launch would not fill the chip."""
from perceiver_io_amd.ops.attention import pick_splits


def test_headline_shapes_unsplit():
    assert pick_splits(64, 4, 256, 512) == 1   # mlm256 cross-attention: 512 four-wave workgroups
    assert pick_splits(64, 4, 256, 256) == 1   # mlm256 self-attention


def test_few_workgroups_split():
    assert pick_splits(8, 4, 512, 8192) == 8   # long-context MLM: 128 workgroups over 8192 keys
    assert pick_splits(4, 4, 32, 16384) > 1    # LArTPC-like: 16 one-wave workgroups over many keys


def test_two_waves_per_cu_short_keys_unsplit():
    # mlm64 cross-attention: 256 two-wave workgroups over 512 keys — the combine costs more
    assert pick_splits(64, 4, 64, 512) == 1
    assert pick_splits(64, 4, 64, 512, dropout=True) == 2


def test_one_wave_per_simd_splits_only_with_dropout():
    # the text classifiers' cross-attention at batch 128: 512 two-wave workgroups
    assert pick_splits(128, 4, 64, 512) == 1
    assert pick_splits(128, 4, 64, 512, dropout=True) == 2
    assert pick_splits(128, 4, 64, 64, dropout=True) == 1  # too few key tiles to split
