class RescaleAction:
    def __init__(self, *a, **k):
        raise NotImplementedError('stub')
