"""The package's evaluator configuration (acs_mi355x/config.py, the product's copy of
cfg/config.json:269-308) equals the oracle's restatement of the same JSON and the
reference's own file."""
import json
import os

from acs_mi355x import config
from oracle import acs_oracle

REF_CFG = "/root/reference/cfg/config.json"


def test_package_config_equals_oracle():
    assert config.SERVICE_URNS == acs_oracle.FULL_URNS
    assert config.CORE_SPEC_URNS == acs_oracle.CORE_SPEC_URNS
    assert config.COMBINING_ALGORITHMS == acs_oracle.DEFAULT_CAS


def test_package_config_equals_reference_file():
    if not os.path.exists(REF_CFG):  # the GPU box has no reference tree
        return
    with open(REF_CFG) as f:
        opts = json.load(f)["policies"]["options"]
    assert opts["urns"] == config.SERVICE_URNS
    assert opts["combiningAlgorithms"] == config.COMBINING_ALGORITHMS
