"""The reference's human_control.py (human_control.py:1-36): ``HumanInput``,
the left-paddle model whose ``run`` returns the held [w, s] keys as [up, down].

The reference reads the keyboard with pynput (human_control.py:26-32).  Here a
key source can also be given, so a game against a network runs headless:
``HumanInput(keys=...)`` takes either a callable ``keys(frame, input_vector)
-> (w, s)`` (``frame`` = 0, 1, ... counts the calls, i.e. the frames on which
get_actions consults the left model, main.py:143-148) or an iterable of (w, s)
pairs (held keys per call; exhausted = nothing held).  Without ``keys`` the
pynput listener of the reference is started when pynput is importable.
"""
button_w = 0
button_s = 1
button_list = [0, 0]  # the keyboard listener's held keys (human_control.py:5-7)


def on_press(key):
    ch = getattr(key, "char", None)
    if ch == 'w':
        button_list[button_w] = 1
    elif ch == 's':
        button_list[button_s] = 1


def on_release(key):
    ch = getattr(key, "char", None)
    if ch == 'w':
        button_list[button_w] = 0
    elif ch == 's':
        button_list[button_s] = 0


class HumanInput:
    """A model with ``run(input_vector) -> [up, down]`` (the duck-typed model
    interface of get_actions, main.py:138-154) driven by held keys."""

    def __init__(self, keys=None):
        self.frame = 0
        self.listener = None
        self._call = self._iter = None
        if keys is None:
            try:
                from pynput import keyboard
            except ImportError as e:  # no keyboard in a headless box: a key source is required
                raise RuntimeError("HumanInput: pynput is not installed; pass keys= (a callable "
                                   "keys(frame, input_vector) -> (w, s) or an iterable of (w, s))") from e
            self.listener = keyboard.Listener(on_press=on_press, on_release=on_release)
            self.listener.start()
        elif callable(keys):
            self._call = keys
        else:
            self._iter = iter(keys)

    def run(self, input_vector=None):
        f = self.frame
        self.frame += 1
        if self._call is not None:
            w, s = self._call(f, input_vector)
        elif self._iter is not None:
            w, s = next(self._iter, (0, 0))
        else:
            w, s = button_list[button_w], button_list[button_s]
        return [int(bool(w)), int(bool(s))]
