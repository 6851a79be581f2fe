"""``python -m relayrl_prototype_amd ...`` -- see runtime/launcher.py."""
import sys

from .runtime.launcher import main

sys.exit(main())
