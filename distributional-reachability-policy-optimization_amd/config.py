"""Typed hierarchical configuration with the reference's semantics (src/config.py:1-160):
class-attribute defaults, JSON-dict ``update`` with type checks, ``Optional``/``Require``
placeholders, dotted ``nested_set`` overrides and ``Configurable`` copying fields onto
the instance. Existing reference JSON configs validate unchanged."""
import copy

SIMPLE_TYPES = {bool, int, float, str}


def _check_list(items):
    for x in items:
        if isinstance(x, list):
            _check_list(x)
        elif type(x) not in SIMPLE_TYPES:
            raise ValueError('Lists in configs can contain only other lists or simple types')


class Require:
    def __init__(self, dtype):
        self.dtype = dtype

    def __repr__(self):
        return f'Require({self.dtype})'


class Optional:
    def __init__(self, dtype):
        self.dtype = dtype

    def __repr__(self):
        return f'Optional({self.dtype})'


class TaggedUnion:
    def __init__(self, **config_classes):
        self.config_classes = config_classes

    def parse(self, d):
        cfg = self.config_classes[d.pop('_tag_')]()
        cfg.update(d)
        return cfg


class BaseConfig:
    def vars(self):
        out = {}
        for key in dir(self):
            if key.startswith('_'):
                continue
            val = getattr(self, key)
            if not callable(val):
                out[key] = val
        return out

    def vars_recursive(self):
        return {k: (v.vars_recursive() if isinstance(v, BaseConfig) else v) for k, v in self.vars().items()}

    def __init__(self, **kwargs):
        fields = self.vars()
        fields.update(kwargs)
        for key, val in fields.items():
            # nested configs are per-instance copies (the class default object is never mutated)
            setattr(self, key, copy.deepcopy(val) if isinstance(val, BaseConfig) else val)

    def typesafe_set(self, key, value):
        assert type(value) in SIMPLE_TYPES
        cur = getattr(self, key)
        if isinstance(cur, Optional):
            expected = cur.dtype
        elif isinstance(cur, Require):
            expected = cur.dtype
        else:
            assert type(cur) in SIMPLE_TYPES
            expected = type(cur)
        assert isinstance(value, expected), f'Got wrong type for key {key}: expected {expected} but got {type(value)}'
        setattr(self, key, value)

    def update(self, d):
        for key, val in d.items():
            assert hasattr(self, key), f'Cannot set non-existent key {key} in {self}'
            if type(val) in SIMPLE_TYPES:
                self.typesafe_set(key, val)
            elif isinstance(val, dict):
                cur = getattr(self, key)
                if isinstance(cur, BaseConfig):
                    cur.update(val)
                elif isinstance(cur, TaggedUnion):
                    setattr(self, key, cur.parse(val))
                elif key == 'env_cfg':
                    setattr(self, key, val)
                else:
                    raise ValueError(f'Given a dict for key {key}, which is not a BaseConfig or TaggedUnion')
            elif isinstance(val, list):
                _check_list(val)
                setattr(self, key, copy.deepcopy(val))
            else:
                raise ValueError(f'Object of unexpected type: {val} ({type(val)})')

    def _nested_set(self, path, value):
        if len(path) == 1:
            if hasattr(self, path[0]):
                self.typesafe_set(path[0], value)
                return True
            return False
        sub = getattr(self, path[0])
        assert isinstance(sub, BaseConfig)
        return sub._nested_set(path[1:], value)

    def nested_set(self, path, value):
        assert isinstance(path, list)
        if not self._nested_set(path, value):
            raise ValueError(f"Cannot override non-existent key {'.'.join(path)}")

    def verify(self):
        for key, val in self.vars().items():
            if isinstance(val, list):
                _check_list(val)
            elif isinstance(val, BaseConfig):
                val.verify()
            elif isinstance(val, Require):
                raise ValueError(f'Required key {key} has not been set')
            elif isinstance(val, Optional):
                setattr(self, key, None)
            elif isinstance(val, TaggedUnion):
                raise ValueError(f'TaggedUnion for key {key} has not been set')
            elif key != 'env_cfg':
                assert type(val) in SIMPLE_TYPES or val is None, f'Invalid value for key {key}: {val}'

    def __str__(self):
        return 'Config(' + ', '.join(f'{k}={v}' for k, v in vars(self).items()) + ')'


class Configurable:
    """Subclasses define a nested ``Config``; its fields are copied onto the instance."""

    def __init__(self, config):
        assert type(config) is self.__class__.Config, f'expected {self.__class__.Config}, got {type(config)}'
        self.config = copy.deepcopy(config)
        for key, val in vars(self.config).items():
            setattr(self, key, val)
