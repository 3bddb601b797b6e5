"""The reference's flag surface for this path: run_job.py:13-48 (user CLI) and
OpenAIGym/parse.py:9-70 (worker flags), reduced to what the learner/predictor hot path and
its single-node launcher (`python -m ba3c_amd.train`) consume.  Slurm / TF-server / Neptune
flags are accepted and ignored."""
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
    p.add_argument("--environment", "-e", "--env", dest="environment", default="Breakout-v0")
    p.add_argument("--channels", type=int, default=1)
    p.add_argument("--num_actions", type=int, default=4)
    p.add_argument("--predict_batch_size", type=int, default=16)
    p.add_argument("--conv_init", default="normal", choices=["normal", "uniform", "xavier"])
    p.add_argument("--fc_init", default="uniform", choices=["normal", "uniform"])
    p.add_argument("--simulator_procs", type=int, default=100)
    p.add_argument("--save_every", type=int, default=0)
    # parse.py worker flags of the training loop
    p.add_argument("--load", default=None)
    p.add_argument("--max_steps", type=int, default=None)
    p.add_argument("--steps_per_epoch", type=int, default=250)
    p.add_argument("--max_epoch", type=int, default=1000)
    p.add_argument("--send_debug_every", type=int, default=100)
    p.add_argument("--dummy", type=int, default=0)
    p.add_argument("--dummy_predictor", type=int, default=0)
    p.add_argument("--models_dir", default="models")
    p.add_argument("--experiment_dir", "--exp_dir", dest="experiment_dir", default=".")
    p.add_argument("--seed", type=int, default=None,
                   help="variable initialiser seed (default: the worker index, train.py:678-679)")
    # accepted for compatibility, no effect on the single-node path
    for name in ("--njobs", "-n", "--cores", "-c", "--nr_towers", "--nr_predict_towers",
                 "--intra_op_par", "--inter_op_par", "--mkl", "--cpu", "--sync", "--queue_size",
                 "--port", "--tf_port", "--threads_to_trace"):
        p.add_argument(name, type=int, default=None, help=argparse.SUPPRESS)
    for name in ("--name", "--tags", "-t", "--log_dir", "--train_log_path", "--gpu", "--early_stopping",
                 "-s", "--task"):
        p.add_argument(name, default=None, help=argparse.SUPPRESS)
    for name in ("--offline", "--intel_tf", "--short", "--debug_charts", "--save_output",
                 "--eval_node", "--record_node", "--schedule_hyper"):
        p.add_argument(name, action="store_true", help=argparse.SUPPRESS)
    return p


def resolve(args):
    """Apply the reference's implicit rules: --use_normal_fc disables replace_with_conv
    (run_job.py:131); --adam_debug sets beta2 := beta1 (train.py:460-461); --use_sync needs
    --ngrads (run_job.py:55-57)."""
    if args.replace_with_conv is None:
        args.replace_with_conv = not args.use_normal_fc
    if args.adam_debug:
        args.beta2 = args.beta1
    if args.use_sync and args.ngrads is None:
        raise SystemExit("if using SyncReplicasOptimizer you have to specify --ngrads argument")
    return args
