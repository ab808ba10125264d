"""Trainer state, control and callback dispatch of the transformers Trainer
that the reference trainers inherit (GRPOTrainer passes `callbacks` to
`Trainer.__init__`, grpo_trainer.py:837-846; PPOTrainer builds its own
CallbackHandler, ppo_trainer.py:264-275).

The loop (`train`) follows transformers' `_inner_training_loop`: on_train_begin,
per optimizer step on_step_begin / on_pre_optimizer_step / on_optimizer_step /
on_step_end, then the `DefaultFlowCallback` decisions (log every
logging_steps, evaluate every eval_steps, save every save_steps, stop and save
at max_steps) merged with whatever the user's callbacks set on the control
object, then on_log / on_evaluate / on_save, and on_train_end.  Callbacks are
given the transformers TrainerState / TrainerControl objects when transformers
is importable (it is in this image), the keyword arguments transformers passes
(`model` is the engine's CausalLM, `optimizer` its FlatAdamW; there is no torch
dataloader or lr_scheduler object: both are None).
"""
from __future__ import annotations

from dataclasses import dataclass

try:  # the objects user callbacks are written against
    from transformers.trainer_callback import TrainerCallback, TrainerControl, TrainerState
except Exception:  # pragma: no cover - transformers is part of the image
    TrainerCallback = object

    @dataclass
    class TrainerControl:  # transformers.trainer_callback.TrainerControl fields
        should_training_stop: bool = False
        should_epoch_stop: bool = False
        should_save: bool = False
        should_evaluate: bool = False
        should_log: bool = False

        def _new_training(self):
            self.should_training_stop = False

        def _new_epoch(self):
            self.should_epoch_stop = False

        def _new_step(self):
            self.should_save = self.should_evaluate = self.should_log = False

    class TrainerState:  # the fields the loops and reward functions read
        def __init__(self, **kw):
            self.epoch, self.global_step, self.max_steps = 0.0, 0, 0
            self.logging_steps, self.eval_steps, self.save_steps = 500, 500, 500
            self.num_input_tokens_seen, self.total_flos = 0, 0.0
            self.log_history: list = []
            self.best_metric = self.best_global_step = self.best_model_checkpoint = None
            self.is_local_process_zero = self.is_world_process_zero = True
            self.is_hyper_param_search = False
            self.trial_name = self.trial_params = None
            self.__dict__.update(kw)

EVENTS = ("on_init_end", "on_train_begin", "on_train_end", "on_epoch_begin", "on_epoch_end", "on_step_begin",
          "on_pre_optimizer_step", "on_optimizer_step", "on_substep_end", "on_step_end", "on_evaluate",
          "on_predict", "on_save", "on_log", "on_prediction_step")


def new_state(rank: int = 0, local_rank: int = 0) -> "TrainerState":
    st = TrainerState()
    st.is_world_process_zero = rank == 0
    st.is_local_process_zero = local_rank == 0
    return st


class CallbackHandler:
    """transformers.trainer_callback.CallbackHandler: calls each event on every
    callback (classes are instantiated), threading one TrainerControl through;
    a callback's non-None return value replaces the control object."""

    def __init__(self, callbacks, trainer):
        self.callbacks: list = []
        self.trainer = trainer
        for cb in callbacks or []:
            self.add_callback(cb)
        self.control = TrainerControl()

    def add_callback(self, callback):
        cb = callback() if isinstance(callback, type) else callback
        self.callbacks.append(cb)

    def pop_callback(self, callback):
        for cb in self.callbacks:
            if (isinstance(callback, type) and isinstance(cb, callback)) or cb is callback:
                self.callbacks.remove(cb)
                return cb
        return None

    def remove_callback(self, callback):
        self.pop_callback(callback)

    # the flags transformers' CallbackHandler clears before dispatching an event
    _RESETS = {"on_train_begin": ("should_training_stop",), "on_epoch_begin": ("should_epoch_stop",),
               "on_step_begin": ("should_log", "should_evaluate", "should_save"), "on_log": ("should_log",),
               "on_evaluate": ("should_evaluate",), "on_save": ("should_save",)}

    def call(self, event: str, **kwargs):
        t = self.trainer
        for flag in self._RESETS.get(event, ()):
            setattr(self.control, flag, False)
        for cb in self.callbacks:
            fn = getattr(cb, event, None)
            if fn is None:
                continue
            out = fn(t.args, t.state, self.control, model=t.model, processing_class=t.processing_class,
                     optimizer=t.optimizer, lr_scheduler=None, train_dataloader=None, eval_dataloader=None, **kwargs)
            if out is not None:
                self.control = out
        return self.control
