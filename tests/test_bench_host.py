"""bench.py's host-side record keeping, on CPU: the amd-smi fields of the box
record (parsed from a metric dump a GPU box wrote in round 3, kept as
tests/data/amd_smi_metric_r03.txt) and
the counter deltas over the timed region."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DUMP = os.path.join(ROOT, 'tests', 'data', 'amd_smi_metric_r03.txt')


def test_smi_fields_parse_a_real_dump():
    import bench
    text = open(DUMP).read()
    got = {}
    for key, pat in bench._SMI_FIELDS:
        m = re.search(pat, text)
        if m:
            got[key] = float(m.group(1))
    assert got['used_vram_mb'] == 225420        # the other tenant's memory, round 3
    assert got['ppt_acc'] == 3788151
    assert got['mem_clk_mhz'] == 2000 and got['fclk_mhz'] == 1250
    assert got['mem_temp_c'] == 34 and got['hotspot_c'] == 47
    assert got['socket_power_w'] == 261


def test_box_state_deltas():
    import bench
    a = {'t': 1.0, 'ppt_acc': 10.0, 'energy_j': 5.0, 'used_vram_mb': 3.0}
    b = {'t': 3.5, 'ppt_acc': 16.0, 'energy_j': 9.0, 'used_vram_mb': 7.0}
    st = bench.box_state(0, a, b, {'store_gbs': 1.0}, {'store_gbs': 2.0})
    assert st['delta'] == {'t': 2.5, 'ppt_acc': 6.0, 'energy_j': 4.0}
    assert st['probe_before'] == {'store_gbs': 1.0}
    assert bench.box_state(0, None, b, None, None) == {'probe_before': None, 'probe_after': None}
