"""State-dict layout of the reference's full-size AFE() and Generator() (models.py:922-945,
1085-1111): {key: shape} lists FROM THE REFERENCE, so that checkpoints of those modules
(logger.py:92-115 save_cpk's 'afe' / 'generator' entries) load into the product modules.

    python tests/golden/make_golden_keys.py      (build container; writes module_keys.json)
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import import_reference  # noqa: E402


def main():
    _, models, _ = import_reference()
    out = {}
    for name, m in (("afe", models.AFE()), ("generator", models.Generator())):
        out[name] = [[k, list(v.shape)] for k, v in m.state_dict().items()]
    with open(os.path.join(HERE, "module_keys.json"), "w") as f:
        json.dump(out, f)
    print({k: len(v) for k, v in out.items()})


if __name__ == "__main__":
    main()
