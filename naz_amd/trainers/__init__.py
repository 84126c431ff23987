from .train_flows import DataParallel, GraphedNllStep, get_params, nll_step, predict, set_params, train, train_lightning

__all__ = ["DataParallel", "GraphedNllStep", "get_params", "nll_step", "predict", "set_params", "train", "train_lightning"]
