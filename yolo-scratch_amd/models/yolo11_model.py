def build_yolo11(*a, **k):
    raise NotImplementedError
