#!/usr/bin/env python3
"""Config 4 (BASELINE.json): A2C on PongSynth-v0 pixels with the Nature CNN on MFMA.
One process per GPU; with --gpus N the launcher spawns torchrun ranks (DP all-reduce).

    python examples/pong_a2c.py --epochs 2000
    python -m relayrl_prototype_amd train --preset pong-a2c --gpus 8 --epochs 2000
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from relayrl_prototype_amd.runtime.launcher import main

if __name__ == "__main__":
    args = sys.argv[1:] or ["--epochs", "200"]
    sys.exit(main(["train", "--preset", "pong-a2c"] + args))
