"""The reference's flag surface for this path: run_job.py:13-48 (user CLI) and
OpenAIGym/parse.py:9-70 (worker flags), reduced to what the learner/predictor hot path
consumes.  Slurm / TF-server / Neptune flags are accepted and ignored."""
import argparse


def string_to_bool(s):        # parse.py:5-6
    return str(s).lower() == "true"


def build_parser():
    p = argparse.ArgumentParser(description="BA3C learner/predictor on MI355X")
    # run_job.py flags
    p.add_argument("--batch_size", "-b", type=int, default=128)
    p.add_argument("--optimizer", "-o", default="adam",
                   choices=["adam", "gd", "adagrad", "adadelta", "momentum", "rms"])
    p.add_argument("--lr", "-l", "--learning_rate", dest="lr", type=float, default=0.00015)
    p.add_argument("--fc_neurons", type=int, default=256)
    p.add_argument("--fc_splits", type=int, default=1)
    p.add_argument("--use_normal_fc", action="store_true")
    p.add_argument("--replace_with_conv", type=string_to_bool, default=None)
    p.add_argument("--ps", type=int, default=1)
    p.add_argument("--use_sync", action="store_true")
    p.add_argument("--ngrads", "-g", "--num_grad", dest="ngrads", type=int, default=None)
    p.add_argument("--epsilon", type=float, default=1e-8)
    p.add_argument("--beta1", type=float, default=0.9)
    p.add_argument("--beta2", type=float, default=0.999)
    p.add_argument("--adam_debug", action="store_true")
    p.add_argument("--environment", "-e", default="Breakout-v0")
    p.add_argument("--channels", type=int, default=1)
    p.add_argument("--num_actions", type=int, default=4)
    p.add_argument("--predict_batch_size", type=int, default=16)
    p.add_argument("--conv_init", default="normal", choices=["normal", "uniform", "xavier"])
    p.add_argument("--fc_init", default="uniform", choices=["normal", "uniform"])
    # accepted for compatibility, no effect on the single-node path
    for name in ("--njobs", "-n", "--cores", "-c", "--simulator_procs"):
        p.add_argument(name, type=int, default=None, help=argparse.SUPPRESS)
    return p


def resolve(args):
    """Apply the reference's implicit rules: --use_normal_fc disables replace_with_conv
    (run_job.py:131); --adam_debug sets beta2 := beta1 (train.py:460-461)."""
    if args.replace_with_conv is None:
        args.replace_with_conv = not args.use_normal_fc
    if args.adam_debug:
        args.beta2 = args.beta1
    if args.use_sync and args.ngrads is None:
        raise SystemExit("if using SyncReplicasOptimizer you have to specify --ngrads argument")
    return args
