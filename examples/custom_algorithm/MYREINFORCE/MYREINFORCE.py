"""A user algorithm plugin: ``TrainingServer("MYREINFORCE", ..., algorithm_dir="examples/custom_algorithm")``
loads ``<algorithm_dir>/MYREINFORCE/MYREINFORCE.py`` and instantiates class ``MYREINFORCE``
(the reference's plugin convention, python_algorithm_reply.py LoadScripts).  Subclass a
built-in to reuse its device kernels and override what you need."""
from relayrl_prototype_amd.algorithms.reinforce import REINFORCE


class MYREINFORCE(REINFORCE):
    CONFIG_NAME = "REINFORCE"  # reuse the REINFORCE block of relayrl_config.json

    def exp_name(self):
        return "my-reinforce"

    def log_epoch(self):
        super().log_epoch()
