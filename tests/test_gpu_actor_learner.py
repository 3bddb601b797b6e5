"""BASELINE configs[0] ("plumbing"): the whole BA3C actor-learner cycle on one GPU with a
synthetic environment — frame history, predictor forward, numpy-exact sampling, n-step
returns, BatchData and the fused learner step — runs end to end, and the datapoints the
learner consumed are the reference simulator master's for the same frames/actions/rewards."""
import numpy as np
import pytest
import torch

from oracle import ba3c_oracle as O

pytestmark = pytest.mark.gpu


def test_actor_learner_runs_and_feeds_the_reference_datapoints():
    from ba3c_amd.actor_learner import ActorLearner
    from ba3c_amd.model import Model
    from ba3c_amd.optimizer import AdamOptimizer
    from ba3c_amd.trainer import Ba3cTrainer, TrainConfig
    E, B = 24, 32
    m = Model(num_actions=4, fc_neurons=128, fc_splits=4, batch_size=B, max_batch=max(B, E))
    m.engine.load_params(O.init_params(128, 4, 4, seed=0, dtype=np.float32))
    tr = Ba3cTrainer(TrainConfig(model=m, optimizer=AdamOptimizer(1e-3, 0.8, 0.75, 1e-8)))
    p0 = m.engine.params.clone()
    loop = ActorLearner(tr, n_envs=E, batch_size=B, seed=1)

    # mirror the simulator master on the host from what the loop's components produce
    mirror = O.SimulatorMasterMirror()
    consumed = []
    orig_put = loop.queue.put

    def put(dps):
        consumed.extend(zip(dps.action.cpu().numpy().tolist(), dps.R.cpu().numpy().tolist()))
        orig_put(dps)
    loop.queue.put = put
    orig_on_state, orig_on_reward = loop.buf.on_state, loop.buf.on_reward

    def on_state(states, actions, values):
        for e, (a, v) in enumerate(zip(actions.cpu().numpy(), values.cpu().numpy())):
            mirror.on_state(e, None, int(a), np.float32(v))
        orig_on_state(states, actions, values)

    def on_reward(rew, over):
        for e, (r, o) in enumerate(zip(rew.cpu().numpy(), over.cpu().numpy())):
            mirror.on_message(e, float(r), bool(o))
        return orig_on_reward(rew, over)
    loop.buf.on_state, loop.buf.on_reward = on_state, on_reward

    loop.run(40)
    torch.cuda.synchronize()
    assert loop.train_steps >= 4
    sc = loop.last_scalars.cpu().numpy()
    assert np.all(np.isfinite(sc))
    assert not torch.equal(m.engine.params, p0)
    want = [(k["action"], float(np.float32(R))) for k, R, _, _ in mirror.queue]
    assert consumed == want and len(want) >= B * loop.train_steps


def test_launcher_runs_sync_training_and_saves_a_checkpoint(tmp_path):
    """`python -m ba3c_amd.train` on the README's best flags (run_job.py -o adam --use_sync
    -b 32 --fc_neurons 128 --fc_splits 4 --beta1 0.8 --beta2 0.75), one GPU = world size 1:
    the actor-learner loop trains 6 steps through SyncReplicasOptimizer's RCCL all-reduce,
    writes the metrics channels and a ModelSaver checkpoint that --load restores."""
    from ba3c_amd.train import main
    argv = ("-o adam --use_sync -g 1 -l 0.001 -b 32 --fc_neurons 128 --fc_splits 4 "
            "--epsilon 1e-8 --beta1 0.8 --beta2 0.75 --simulator_procs 64 --max_steps 6 "
            "--send_debug_every 3 --save_every 6").split()
    argv += ["--models_dir", str(tmp_path / "models"), "--experiment_dir", str(tmp_path / "exp")]
    out = main(argv)
    assert out["global_step"] >= 6 and out["last"] is not None
    assert np.isfinite(out["last"]["cost"])
    ckpts = list((tmp_path / "models").rglob("*.npz"))
    assert len(ckpts) == 1
    with np.load(str(ckpts[0]), allow_pickle=False) as f:
        assert "conv0/W" in f.files and "conv0/W/Adam" in f.files and int(f["global_step"]) == 6
    assert any((tmp_path / "exp").iterdir())
    out2 = main(argv[:-4] + ["--max_steps", "8", "--load", str(ckpts[0]),
                             "--models_dir", str(tmp_path / "m2"), "--experiment_dir", str(tmp_path / "e2")])
    assert out2["global_step"] >= 8
