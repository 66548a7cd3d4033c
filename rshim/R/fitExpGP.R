# FitOCTLib::fitExpGP and FitOCTLib::fitMonoExp with the MI355X engine behind them
# (SURVEY.md §8b, §8f rows 1-3).  Signatures and return values as called at
# FitOCT.R:95,110-124, priPost.R:2-16 and server.R:341-343,408-426; extra arguments are
# optional.  Every method runs on the GPU through the .Call entries of src/fitoct_R.c:
#   'sample' -> one Stan CSV per chain (fitoct_write_stan_csv) -> rstan::read_stan_csv
#   'optim'  -> rstan::optimizing(as_vector = FALSE, hessian = TRUE)-shaped list
#   'vb'     -> CmdStan variational CSV (fitoct_write_vb_csv) -> rstan::read_stan_csv
# backend = 'rstan' delegates to the original FitOCTLib functions.

fitoct_device_count <- function() .Call(fitoct_R_device_count)

# n_gpus GPUs from `device` on (n_gpus = NA: every visible GPU from `device` on)
fitoct_devices <- function(device, n_gpus) {
  if (is.na(n_gpus)) n_gpus <- max(1L, fitoct_device_count() - as.integer(device))
  if (n_gpus < 1 || n_gpus > 16) stop('fitExpGP: n_gpus must be in 1..16')
  as.integer(device) + seq_len(as.integer(n_gpus)) - 1L
}

# GP control grid (server.R:623-631)
fitoct_xGP <- function(Nn, gridType) {
  if (gridType == 'internal') {
    dx <- 1 / (Nn + 1)
    seq(dx / 2, 1 - dx / 2, length.out = Nn)
  } else {
    seq(0, 1, length.out = Nn)
  }
}

fitoct_problem <- function(x, y, uy, dataType, Nn, gridType, rho_scale, theta0, Sigma0,
                           prior, lambda_rate = 0.1, lambda_scale = 10, nu = 1, prior_PD = 0)
  list(x = as.double(x), y = as.double(y), uy = as.double(uy),
       dataType = as.integer(dataType), Nn = as.integer(Nn),
       gridType = as.character(gridType), rho = as.double(rho_scale),
       theta0 = as.double(theta0), Sigma0 = as.double(Sigma0), prior = as.integer(prior),
       lambda_rate = as.double(lambda_rate), lambda_scale = as.double(lambda_scale),
       nu = as.double(nu), prior_PD = as.integer(prior_PD))

# sampling: stdout gets rstan-format "Chain k: Iteration: ..." lines (the Shiny server
# parses them from its stan.log sink, server.R:391-393,457-484)
# devices: GPU ordinals; the library splits the chains over them (one host thread per
# GPU), which replaces options(mc.cores = parallel::detectCores()) (FitOCT.R:13, server.R:19)
# Up to `csv_max_chains` chains the fit goes through one CmdStan CSV per chain and
# rstan::read_stan_csv (the stanfit rstan itself builds); above it (config 4: 8192 chains
# of 1500 rows) the draws come back from .Call as one binary array and fitoct_stanfit
# assembles the same stanfit object without any text round trip.
fitoct_sample <- function(prob, nb_chains, nb_warmup, nb_iter, seed, adapt_delta,
                          max_treedepth, devices, csv_max_chains = 64L) {
  ctrl <- list(chains = as.integer(nb_chains), warmup = as.integer(nb_warmup),
               samples = as.integer(nb_iter - nb_warmup), seed = as.double(seed),
               adapt_delta = as.double(adapt_delta), max_treedepth = as.integer(max_treedepth),
               devices = as.integer(devices))
  if (nb_chains > csv_max_chains)
    return(fitoct_stanfit(.Call(fitoct_R_sample_bulk, prob, ctrl), ctrl))
  files <- vapply(seq_len(nb_chains), function(i) tempfile(fileext = '.csv'), character(1))
  on.exit(unlink(files))
  .Call(fitoct_R_sample, prob, ctrl, files)
  rstan::read_stan_csv(files)
}

# A stanfit from fitoct_R_sample_bulk's arrays, assembled as rstan::read_stan_csv assembles
# it from CmdStan CSV files (the same sim slot: per-chain named draw vectors with the
# sampler_params / adaptation_info / elapsed_time / args attributes, warmup2, n_save,
# permutation), so print(), extract(), as.matrix(), summary(), traceplot(inc_warmup = TRUE)
# and get_sampler_params() read it as they read the CSV route's fit (plotExpGP.R:7-44,
# server.R:88-237).  res$draws: array [rows, 7 + n_params, chains], warmup rows first.
fitoct_stanfit <- function(res, ctrl, model_name = 'ExpGP') {
  d <- res$draws
  rows <- dim(d)[1]
  chains <- dim(d)[3]
  cols <- dimnames(d)[[2]]
  lead <- cols[1:7]                                   # lp__, then the 6 sampler columns
  par_cols <- cols[-(1:7)]
  flat <- sub('\\.([0-9]+)$', '[\\1]', par_cols)      # theta.1 -> theta[1] (Stan's flatnames)
  base <- sub('\\[[0-9]+\\]$', '', flat)
  pars_oi <- c(unique(base), 'lp__')
  dims_oi <- c(lapply(unique(base), function(b) {
    n <- sum(base == b)
    if (n == 1 && !grepl('\\[', flat[match(b, base)])) integer(0) else n
  }), list(integer(0)))
  names(dims_oi) <- pars_oi
  fnames_oi <- c(flat, 'lp__')
  warmup2 <- ctrl$warmup                              # save_warmup: warmup rows are kept
  n_kept <- rows - warmup2
  samples <- lapply(seq_len(chains), function(k) {
    m <- d[, , k]
    draws <- c(lapply(seq_along(par_cols), function(j) m[, 7 + j]), list(m[, 1]))
    names(draws) <- fnames_oi
    sp <- as.data.frame(m[, 2:7, drop = FALSE])
    names(sp) <- lead[2:7]
    attr(draws, 'sampler_params') <- sp
    attr(draws, 'adaptation_info') <- paste0(
      '# Adaptation terminated\n# Step size = ', format(res$stepsize[k], digits = 8),
      '\n# Diagonal elements of inverse mass matrix:\n# ',
      paste(format(res$inv_metric[, k], digits = 8), collapse = ', '), '\n')
    attr(draws, 'elapsed_time') <- c(warmup = res$elapsed[1, k], sample = res$elapsed[2, k])
    post <- if (n_kept > 0) (warmup2 + 1):rows else integer(0)
    attr(draws, 'mean_pars') <- vapply(draws[seq_along(par_cols)],
                                       function(v) mean(v[post]), numeric(1))
    attr(draws, 'mean_lp__') <- mean(m[post, 1])
    attr(draws, 'args') <- list(sampler_t = 'NUTS(diag_e)', chain_id = k, iter = rows,
                                warmup = warmup2, thin = 1L, seed = ctrl$seed,
                                method = 'sampling', save_warmup = TRUE,
                                control = list(adapt_delta = ctrl$adapt_delta,
                                               max_treedepth = ctrl$max_treedepth))
    draws
  })
  sim <- list(samples = samples, iter = rows, thin = 1L, warmup = warmup2, chains = chains,
              n_save = rep(rows, chains), warmup2 = rep(warmup2, chains),
              permutation = lapply(seq_len(chains), function(k) sample.int(n_kept)),
              pars_oi = pars_oi, dims_oi = dims_oi, fnames_oi = fnames_oi,
              n_flatnames = length(fnames_oi))
  stan_args <- lapply(seq_len(chains), function(k) attr(samples[[k]], 'args'))
  null_dso <- new('cxxdso', sig = list(character(0)), dso_saved = FALSE,
                  dso_filename = character(0), modulename = character(0),
                  system = R.version$system, cxxflags = character(0),
                  .CXXDSOMISC = new.env(parent = emptyenv()))
  null_sm <- new('stanmodel', model_name = model_name, model_code = character(0),
                 model_cpp = list(), dso = null_dso)
  new('stanfit', model_name = model_name, model_pars = pars_oi, par_dims = dims_oi,
      mode = 0L, sim = sim, inits = list(), stan_args = stan_args, stanmodel = null_sm,
      date = date(), .MISC = new.env(parent = emptyenv()))
}

# rstan::optimizing(as_vector = FALSE, hessian = TRUE): par grouped by base name
# (fit$par$theta, fit$par$yGP, fit$par$lambda, fit$par$sigma, fit$par$br) plus the
# generated m, resid, dL; hessian on the unconstrained scale with 'theta.1'-style
# dimnames (server.R:114-126,156-172 take sqrt(-1/H[p,p]) after gsub('\\.', '', ...))
fitoct_optimize <- function(prob, device) {
  res <- .Call(fitoct_R_optimize, prob, list(device = as.integer(device), hessian = TRUE))
  base <- sub('\\.[0-9]+$', '', names(res$par))
  par <- lapply(split(unname(res$par), factor(base, levels = unique(base))), identity)
  par$m <- res$m
  par$resid <- res$resid
  if (!is.null(res$dL)) par$dL <- res$dL
  list(par = par, value = res$value, return_code = res$return_code, hessian = res$hessian)
}

fitoct_vb <- function(prob, seed, device) {
  f <- tempfile(fileext = '.csv')
  on.exit(unlink(f))
  .Call(fitoct_R_vb, prob, list(seed = as.double(seed), device = as.integer(device)), f)
  rstan::read_stan_csv(f)
}

fitExpGP <- function(x, y, uy, dataType = 2, Nn = 10, gridType = 'internal',
                     method = 'sample', theta0, Sigma0, lambda_rate = 0.1,
                     rho_scale = 0, nb_warmup = 500, nb_iter = 1000, prior_PD = 0,
                     open_progress = FALSE, nb_chains = 4,
                     prior_type = c('normal', 'lasso', 'horseshoe'),
                     lambda_scale = 10, nu = 1, adapt_delta = 0.8, max_treedepth = 10,
                     seed = sample.int(.Machine$integer.max, 1),
                     backend = c('hip', 'rstan'), device = 0L, n_gpus = 1L) {
  backend <- match.arg(backend)
  prior_type <- match.arg(prior_type)
  if (backend == 'rstan')
    return(FitOCTLib::fitExpGP(x = x, y = y, uy = uy, dataType = dataType, Nn = Nn,
                               gridType = gridType, method = method, theta0 = theta0,
                               Sigma0 = Sigma0, lambda_rate = lambda_rate,
                               rho_scale = rho_scale, nb_warmup = nb_warmup,
                               nb_iter = nb_iter, prior_PD = prior_PD,
                               open_progress = open_progress))
  devices <- fitoct_devices(device, n_gpus)   # after the rstan return: no HIP call for it
  prob <- fitoct_problem(x, y, uy, dataType, Nn, gridType, rho_scale, theta0, Sigma0,
                         match(prior_type, c('normal', 'lasso', 'horseshoe')) - 1L,
                         lambda_rate, lambda_scale, nu, prior_PD)
  fit <- switch(method,
    sample = fitoct_sample(prob, nb_chains, nb_warmup, nb_iter, seed, adapt_delta,
                           max_treedepth, devices),
    optim = fitoct_optimize(prob, device),
    vb = fitoct_vb(prob, seed, device),
    stop("fitExpGP: method must be 'sample', 'optim' or 'vb'"))
  list(fit = fit, method = method, xGP = fitoct_xGP(Nn, gridType), prior_PD = prior_PD,
       lasso = prior_type == 'lasso')
}

# FitOCTLib::fitMonoExp (FitOCT.R:95-97, server.R:341-343): y = theta1 + theta2
# exp(-c x / theta3), flat prior on theta > 0 (⚑ the restated model of include/fitoct.h).
# Returns list(fit, method, best.theta, cor.theta).
fitMonoExp <- function(x, y, uy, dataType = 2, method = 'optim', nb_warmup = 500,
                       nb_iter = 1500, nb_chains = 4,
                       seed = sample.int(.Machine$integer.max, 1),
                       backend = c('hip', 'rstan'), device = 0L, n_gpus = 1L) {
  backend <- match.arg(backend)
  if (backend == 'rstan')
    return(FitOCTLib::fitMonoExp(x = x, y = y, uy = uy, dataType = dataType))
  devices <- fitoct_devices(device, n_gpus)
  theta0 <- .Call(fitoct_R_mono_theta0, as.double(x), as.double(y), as.integer(dataType))
  prob <- fitoct_problem(x, y, uy, dataType, 2L, 'extremal', 0, theta0, diag(3), 3L)
  if (method == 'sample') {
    fit <- fitoct_sample(prob, nb_chains, nb_warmup, nb_iter, seed, 0.8, 10, devices)
    th <- as.matrix(fit, pars = 'theta')
    return(list(fit = fit, method = method, best.theta = colMeans(th), cor.theta = cor(th)))
  }
  if (method != 'optim') stop("fitMonoExp: method must be 'optim' or 'sample'")
  fit <- fitoct_optimize(prob, device)
  theta <- fit$par$theta
  cov_q <- solve(-fit$hessian)                 # unconstrained (log theta) scale
  cov <- cov_q * outer(theta, theta)           # delta method back to theta
  list(fit = fit, method = method, best.theta = theta, cor.theta = cov2cor(cov))
}
