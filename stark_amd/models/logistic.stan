// Bayesian logistic regression, flat priors (Stan User's Guide form).
data {
  int<lower=0> N;
  int<lower=0> K;
  matrix[N, K] x;
  int<lower=0, upper=1> y[N];
}
parameters {
  real alpha;
  vector[K] beta;
}
model {
  y ~ bernoulli_logit(alpha + x * beta);
}
