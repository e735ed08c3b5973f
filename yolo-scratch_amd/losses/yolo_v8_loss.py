class v8DetectionLoss:
    pass
