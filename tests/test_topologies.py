"""Shipped pool topologies (distributed_llm_amd/data/topologies/*.json) parse, name both tiers and
only known model architectures (the reference-model-pair file drives scripts/legacy_ref_models.py)."""
import glob
import os

import pytest

from distributed_llm_amd.config import LARGE, SMALL, canonical_tier, load_config_file
from distributed_llm_amd.models.configs import get_model_config as get_config

TOPO_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "distributed_llm_amd", "data",
                        "topologies")


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(TOPO_DIR, "*.json"))))
def test_topology_file(path):
    spec = {k: v for k, v in load_config_file(path).items() if not k.startswith("_")}   # "_comment"
    assert {canonical_tier(k) for k in spec} == {SMALL, LARGE}
    for s in spec.values():
        if s.get("kind", "engine") in ("engine", "supervised"):
            assert get_config(s["model"]).name
            assert int(s["max_new_tokens"]) > 0


def test_reference_pair_matches_reference_devices():
    """phi3-mini greedy on the small tier, Llama-3-8B sampled on the large tier
    (src/devices/nano_api.py:15-21, orin_api.py:17-18)."""
    spec = load_config_file(os.path.join(TOPO_DIR, "reference_models_1gpu.json"))
    tiers = {canonical_tier(k): v for k, v in spec.items()}
    assert get_config(tiers[SMALL]["model"]).name == "phi3-mini" and tiers[SMALL]["temperature"] == 0.0
    assert get_config(tiers[LARGE]["model"]).name == "llama-3-8b" and tiers[LARGE]["temperature"] > 0
