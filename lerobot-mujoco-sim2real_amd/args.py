"""Hot-path subset of the reference's ``Args`` (``args.py:3-122``).

Only the fields the data-collection and MPC-tracking paths read are kept (SURVEY.md §2 marks
the training fields out of scope): sample/step counts (``args.py:27-34``),
``x_dim``/``u_dim`` (``:47-50``), ``device`` (``:70``), the scene path
(``:91``), the ``.npy`` cache paths (``:97-100``) and the Koopman-MPC fields the batched
controller reads (``model`` :13, ``MPC_type`` :75, ``layers`` :103).  ``__getattr__`` passes
through to the parsed namespace as the reference does (``:120-122``).
"""
import argparse
import os

from .mjcf import SCENE_XML


class Args:
    def __init__(self, argv=None):
        self.parser = argparse.ArgumentParser(description="SO-ARM101 batched data collection")
        p = self.parser
        p.add_argument("--env", type=str, default="SOARM101")
        p.add_argument("--seed", type=int, default=42)
        p.add_argument("--train_samples", type=int, default=50000)
        p.add_argument("--train_steps", type=int, default=20)
        p.add_argument("--test_samples", type=int, default=2000)
        p.add_argument("--test_steps", type=int, default=200)
        p.add_argument("--test_type", type=str, default="all", choices=["sin", "random", "chirp", "all"])
        p.add_argument("--x_dim", type=int, default=8)
        p.add_argument("--u_dim", type=int, default=5)
        p.add_argument("--batch_size", type=int, default=128)
        p.add_argument("--eval_batch_size", type=int, default=128)
        p.add_argument("--device", type=str, default="cuda", choices=["cpu", "cuda"])
        p.add_argument("--data_root", type=str, default=os.path.abspath("."))
        # Koopman-MPC tracking: model kind (:13), MPC form (:75)
        p.add_argument("--model", type=str, default="DKUC", choices=["DKUC", "DBKN"])
        p.add_argument("--MPC_type", type=str, default="delta_mpc", choices=["mpc", "delta_mpc"])
        p.add_argument("--u_z", action="store_true", default=False)  # DBKN kron order (:43)
        self.args = p.parse_args([] if argv is None else argv)
        self.process_args()

    def process_args(self):
        a = self.args
        a.xml_path = SCENE_XML
        a.data_dir_save = os.path.join(a.data_root, a.env, "data")
        a.data_dir_load_train = os.path.join(a.data_dir_save, f"train_data_{a.train_samples}_{a.train_steps}.npy")
        a.data_dir_load_test = os.path.join(
            a.data_dir_save, f"test_data_{a.test_type}_{a.test_samples}_{a.test_steps}.npy")
        a.data_dir_load_val = os.path.join(a.data_dir_save, f"val_data_{a.test_samples}_{a.test_steps}.npy")
        a.layers = [a.x_dim, 64, 64, 64, 64, 24]  # Koopman encoder widths (:103)

    def __getattr__(self, name):
        return getattr(self.args, name)
