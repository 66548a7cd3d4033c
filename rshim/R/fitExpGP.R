# FitOCTLib::fitExpGP with the MI355X sampler behind it (SURVEY.md §8b).
# Signature and return value as called at FitOCT.R:110-124, priPost.R:2-16 and
# server.R:408-426; extra arguments are optional.  method = 'sample' runs on the GPU
# through .Call('fitoct_R_sample') (src/fitoct_R.c); other methods, and
# backend = 'rstan', delegate to the original FitOCTLib function.

fitoct_device_count <- function() .Call(fitoct_R_device_count)

# GP control grid (server.R:623-631)
fitoct_xGP <- function(Nn, gridType) {
  if (gridType == 'internal') {
    dx <- 1 / (Nn + 1)
    seq(dx / 2, 1 - dx / 2, length.out = Nn)
  } else {
    seq(0, 1, length.out = Nn)
  }
}

# one Stan CSV per chain -> rstan::read_stan_csv (a real stanfit: print, extract,
# as.matrix, summary()$summary with Rhat / n_eff, traceplot(inc_warmup = TRUE), pairs)
fitoct_stanfit <- function(res, nb_chains, nb_warmup, nb_iter) {
  ncols <- length(res[[2]])
  arr <- array(res[[1]], dim = c(ncols, nb_iter, nb_chains))   # C order: dims reversed
  files <- vapply(seq_len(nb_chains), function(ch) {
    f <- tempfile(fileext = '.csv')
    writeLines(c('# model = ExpGP', '# method = sample (Default)',
                 sprintf('#   num_samples = %d', nb_iter - nb_warmup),
                 sprintf('#   num_warmup = %d', nb_warmup),
                 '#   save_warmup = 1', '#   thin = 1',
                 sprintf('# Step size = %.17g', res[[3]][ch]),
                 paste(res[[2]], collapse = ',')), f)
    utils::write.table(t(arr[, , ch]), f, sep = ',', append = TRUE,
                       col.names = FALSE, row.names = FALSE)
    f
  }, character(1))
  on.exit(unlink(files))
  rstan::read_stan_csv(files)
}

fitExpGP <- function(x, y, uy, dataType = 2, Nn = 10, gridType = 'internal',
                     method = 'sample', theta0, Sigma0, lambda_rate = 0.1,
                     rho_scale = 0, nb_warmup = 500, nb_iter = 1000, prior_PD = 0,
                     open_progress = FALSE, nb_chains = 4,
                     prior_type = c('normal', 'lasso', 'horseshoe'),
                     lambda_scale = 10, nu = 1, adapt_delta = 0.8, max_treedepth = 10,
                     seed = sample.int(.Machine$integer.max, 1),
                     backend = c('hip', 'rstan'), device = 0L) {
  backend <- match.arg(backend)
  prior_type <- match.arg(prior_type)
  if (backend == 'rstan' || method != 'sample')
    return(FitOCTLib::fitExpGP(x = x, y = y, uy = uy, dataType = dataType, Nn = Nn,
                               gridType = gridType, method = method, theta0 = theta0,
                               Sigma0 = Sigma0, lambda_rate = lambda_rate,
                               rho_scale = rho_scale, nb_warmup = nb_warmup,
                               nb_iter = nb_iter, prior_PD = prior_PD,
                               open_progress = open_progress))
  res <- .Call(fitoct_R_sample, as.double(x), as.double(y), as.double(uy),
               as.integer(dataType), as.integer(Nn), as.character(gridType),
               as.double(rho_scale), as.double(theta0), as.double(Sigma0),
               match(prior_type, c('normal', 'lasso', 'horseshoe')) - 1L,
               as.double(c(lambda_rate, lambda_scale, nu)), as.integer(prior_PD),
               as.integer(nb_chains), as.integer(nb_warmup),
               as.integer(nb_iter - nb_warmup), as.double(seed),
               as.double(adapt_delta), as.integer(max_treedepth),
               as.logical(open_progress), as.integer(device))
  fit <- fitoct_stanfit(res, nb_chains, nb_warmup, nb_iter)
  list(fit = fit, method = method, xGP = fitoct_xGP(Nn, gridType), prior_PD = prior_PD,
       lasso = prior_type == 'lasso')
}
