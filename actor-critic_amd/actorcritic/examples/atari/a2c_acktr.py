"""A2C / ACKTR on Atari — the reference entry point (actorcritic/examples/atari/a2c_acktr.py)
on the MI355X engine.  The structure is the reference's line for line: environments ->
MultiEnv -> AtariModel -> MultiEnvAgent -> A2CObjective -> optimizer ->
``optimize_shared`` -> a session loop that interacts and runs the optimize op.  The
differences are the imports (no tensorflow / kfac / gym) and the synthetic batched
Atari stepper in place of ALE subprocesses.
"""

import os

import numpy as np

import actorcritic.envs.atari.wrappers as wrappers
from actorcritic import checkpoint, parallel
from actorcritic.agents import MultiEnvAgent
from actorcritic.envs.atari.model import AtariModel
from actorcritic.kfac_utils import ColdStartPeriodicInvUpdateKfacOpt, LayerCollection
from actorcritic.multi_env import MultiEnv
from actorcritic.nn import ClipGlobalNormOptimizer, MomentumOptimizer, RMSPropOptimizer, linear_decay
from actorcritic.objectives import A2CObjective
from actorcritic.session import Session, get_or_create_global_step, no_op


def train_a2c_acktr(acktr, env_id, num_envs, num_steps, checkpoint_path, model_name, summary_path=None,
                    max_updates=None, seed=0, log_every=10):
    """Trains an Atari model with A2C (RMSProp, conv3 64) or ACKTR (K-FAC, conv3 32).

    ``num_envs`` is per GPU; with WORLD_SIZE > 1 (torchrun) every rank steps its own shard.
    """
    parallel.init_from_env()
    multi_env = MultiEnv(create_environments(env_id, num_envs, seed=seed))

    conv3_num_filters = 32 if acktr else 64
    model = AtariModel(multi_env.observation_space, multi_env.action_space, conv3_num_filters, random_seed=seed)
    agent = MultiEnvAgent(multi_env, model, num_steps)
    objective = A2CObjective(model, discount_factor=0.99, entropy_regularization_strength=0.01)

    global_step = get_or_create_global_step()
    # 1e7 env-steps (4e7 frames) over the whole job; global steps = env-steps / batch
    max_step = 10000000 / (num_envs * num_steps * parallel.world_size())
    if acktr:
        learning_rate = linear_decay(0.25, 0.025, global_step, max_step, name='learning_rate')
    else:
        learning_rate = linear_decay(0.0007, 0.00007, global_step, max_step, name='learning_rate')

    optimizer = create_optimizer(acktr, model, learning_rate)
    optimize_op = objective.optimize_shared(optimizer, baseline_loss_weight=0.5, global_step=global_step)

    summary_writer = checkpoint.ScalarLog(summary_path) if (summary_path and parallel.rank() == 0) else None
    summary_op = no_op()

    with Session() as session:
        load_model(checkpoint_path, model, optimizer, global_step)
        step = global_step.value
        updates = 0
        try:
            while step < max_step and (max_updates is None or updates < max_updates):
                observations, actions, rewards, terminals, next_observations, infos = agent.interact(session)
                episode_rewards = wrappers.EpisodeInfoWrapper.get_episode_rewards_from_info_batch(infos) \
                    if summary_writer is not None else None

                fetches = [summary_op, global_step, optimize_op]
                if summary_writer is not None and step % log_every == 0:
                    fetches += [objective.policy_loss, objective.baseline_loss, objective.mean_entropy]
                out = session.run(fetches, feed_dict={
                    model.observations_placeholder: observations,
                    model.bootstrap_observations_placeholder: next_observations,
                    model.actions_placeholder: actions,
                    model.rewards_placeholder: rewards,
                    model.terminals_placeholder: terminals,
                }, host=len(fetches) > 3)
                step = global_step.value
                updates += 1
                if len(out) > 3:
                    mean_episode_reward = (np.nan if np.all(np.isnan(episode_rewards))
                                           else float(np.nanmean(episode_rewards)))
                    summary_writer.add(step, policy_loss=float(out[3]), baseline_loss=float(out[4]),
                                       policy_entropy=float(out[5]), episode_reward=mean_episode_reward)
                if step % 100 == 0 and step > 0 and parallel.rank() == 0:
                    save_model(checkpoint_path, model_name, step, model, optimizer)
        except KeyboardInterrupt:
            print('Stop requested')
            if parallel.rank() == 0:
                save_model(checkpoint_path, model_name, step, model, optimizer)
        finally:
            multi_env.close()
            if summary_writer is not None:
                summary_writer.close()
    return model, optimizer


def create_environments(env_id, num_envs, seed=0):
    """The batched synthetic Atari stepper for this rank's env shard."""
    return wrappers.SyntheticAtariEnvs(num_envs, num_actions=wrappers.num_actions_for(env_id), seed=seed,
                                       env_offset=parallel.rank() * num_envs)


def create_optimizer(acktr, model, learning_rate):
    """ACKTR: cold-start Momentum(3e-4, .9)+clip .5 for 30 updates, then K-FAC
    (invert every 10, EMA .99, damping .01, momentum .9, trust region 1e-4);
    A2C: RMSProp + clip .5 (a2c_acktr.py:218-253)."""
    if acktr:
        layer_collection = LayerCollection()
        model.register_layers(layer_collection)
        model.register_predictive_distributions(layer_collection)
        cold_optimizer = MomentumOptimizer(learning_rate=0.0003, momentum=0.9)
        cold_optimizer = ClipGlobalNormOptimizer(cold_optimizer, clip_norm=0.5)
        return ColdStartPeriodicInvUpdateKfacOpt(
            num_cold_updates=30, cold_optimizer=cold_optimizer, invert_every=10, learning_rate=learning_rate,
            cov_ema_decay=0.99, damping=0.01, layer_collection=layer_collection, momentum=0.9,
            norm_constraint=0.0001)
    optimizer = RMSPropOptimizer(learning_rate=learning_rate)
    return ClipGlobalNormOptimizer(optimizer, clip_norm=0.5)


def load_model(checkpoint_path, model, optimizer, global_step):
    path = checkpoint.latest(checkpoint_path)
    if path is None:
        print('No model loaded')
        return False
    checkpoint.load(path, model, optimizer, global_step)
    print('Loaded model')
    return True


def save_model(checkpoint_path, model_name, step, model, optimizer):
    checkpoint.save(os.path.join(checkpoint_path, model_name), step, model, optimizer)
    print('Saved model (step {})'.format(step))


if __name__ == '__main__':
    acktr = True
    env_id = 'BreakoutNoFrameskip-v4'
    num_envs = 32
    num_steps = 20
    results_path = os.path.abspath('./results')
    checkpoint_path = results_path + '/checkpoints/' + env_id
    summary_path = results_path + '/summaries/' + env_id
    os.makedirs(checkpoint_path, exist_ok=True)
    os.makedirs(summary_path, exist_ok=True)
    train_a2c_acktr(acktr, env_id, num_envs, num_steps, checkpoint_path, 'Atari-' + env_id, summary_path)
