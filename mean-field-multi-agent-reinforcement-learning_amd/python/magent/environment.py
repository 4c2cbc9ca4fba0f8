"""Abstract environment interface (reference python/magent/environment.py)."""


class Environment:
    def __init__(self):
        pass

    def reset(self):
        raise NotImplementedError

    def get_observation(self, handle):
        raise NotImplementedError

    def set_action(self, handle, actions):
        raise NotImplementedError

    def step(self):
        raise NotImplementedError

    def render(self):
        raise NotImplementedError

    def render_next_file(self):
        raise NotImplementedError

    def get_reward(self, handle):
        raise NotImplementedError

    def get_num(self, handle):
        raise NotImplementedError

    def get_action_space(self, handle):
        raise NotImplementedError

    def get_view_space(self, handle):
        raise NotImplementedError

    def get_feature_space(self, handle):
        raise NotImplementedError
