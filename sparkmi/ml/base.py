"""pyspark.ml base abstractions: Transformer, Estimator, Model, Evaluator, Pipeline.

Reference flow (mllib_multilayer_perceptron_classifier.py:35-48):
``trainer = MultilayerPerceptronClassifier(...); model = trainer.fit(train);
result = model.transform(test); evaluator.evaluate(result.select("prediction", "label"))``.
"""
from .param import Params


class Transformer(Params):
    def transform(self, dataset, params=None):
        if params:
            return self.copy(params)._transform(dataset)
        return self._transform(dataset)

    def _transform(self, dataset):
        raise NotImplementedError


class Model(Transformer):
    pass


class Estimator(Params):
    def fit(self, dataset, params=None):
        if isinstance(params, (list, tuple)):
            return [self.fit(dataset, p) for p in params]
        if params:
            return self.copy(params)._fit(dataset)
        return self._fit(dataset)

    def _fit(self, dataset):
        raise NotImplementedError


class Evaluator(Params):
    def evaluate(self, dataset, params=None):
        if params:
            return self.copy(params)._evaluate(dataset)
        return self._evaluate(dataset)

    def _evaluate(self, dataset):
        raise NotImplementedError

    def isLargerBetter(self):
        return True


class Pipeline(Estimator):
    def __init__(self, stages=None):
        super().__init__()
        self.stages = list(stages or [])

    def setStages(self, stages):
        self.stages = list(stages)
        return self

    def getStages(self):
        return self.stages

    def _fit(self, dataset):
        fitted = []
        df = dataset
        last_est = max([i for i, s in enumerate(self.stages) if isinstance(s, Estimator)], default=-1)
        for i, st in enumerate(self.stages):
            if isinstance(st, Estimator):
                m = st.fit(df)
                fitted.append(m)
                if i < last_est:
                    df = m.transform(df)
            else:
                fitted.append(st)
                if i < last_est:
                    df = st.transform(df)
        return PipelineModel(fitted)


class PipelineModel(Model):
    def __init__(self, stages):
        super().__init__()
        self.stages = stages

    def _transform(self, dataset):
        for st in self.stages:
            dataset = st.transform(dataset)
        return dataset
